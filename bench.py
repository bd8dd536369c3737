#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the batched hedging env on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--envs E]
                    [--mode rollout|graph|eager]

Workload = BASELINE.json configs[1]: 65,536 parallel envs per GPU, GBM price
advance (Philox4x32-10 normals), Black-Scholes rolling-ATM marks, v2 env with
the train_ppo_v2.py reward settings (abs loss, w=1e-3, lambda=1e-4,
theta=2e-4, 1 bp slippage).  One "step" = one env-step of every env: actions
[N,2] in (pre-generated, HBM-resident), obs [N,13] / reward [N] / done flags
out, auto-reset inside the kernel, plus the market generation of that step.

Modes: `rollout` (default) fuses 64 steps per launch (he_rollout: actions
[64,N,2] in, obs [64,N,13] / reward / terminated out, the collect_rollouts
inner loop of train_ppo_v2.py:48 with actions supplied up front); `graph`
replays he_step launches captured into hipGraphs, one kernel per step (the
Gym step API path); `eager` calls he_step from Python every step.  At N=1 the
JSON line also carries the graph-mode he_step measurement under "step_api".
For N>1 the script runs under torch.distributed.run, one rank per GPU (weak
scaling: E envs per rank, env ids offset by rank), and all-gathers the per-env
episode summaries {return, sum P&L, sum cost, length} (he_episode_summaries) over
RCCL every 256 steps (the rollout-buffer boundary of train_ppo_v2.py:48).
`--gpus N` without WORLD_SIZE in the environment makes this process the launcher:
it runs the PMC pass and the CPU baseline (no GPU call of its own: the PMC pass is a
rocprofv3 child), then starts `python -m torch.distributed.run --nproc-per-node N
bench.py ...` as a child process and exits with its status; rank 0 merges the
launcher's results into its JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Algorithmic HBM bytes, SURVEY.md 8(d) -- the figure roofline.achieved is priced on:
#   he_rollout (fused K-step rollout): 66 B per env-step (action 8 + obs 52 + reward 4 +
#       terminated/truncated 2) + 120 B per env per launch (state read + written, 2 x 60)
#   he_step (Gym API, one launch per step): 186 B per env-step
SURVEY_ROLLOUT_B, SURVEY_ROLLOUT_STATE_B, SURVEY_STEP_B = 66, 120, 186
# What the kernels themselves must move:
#   lds_rollout_kernel (he_rollout, GBM, no book; the market is made in LDS): per env-step
#       action 8 + obs 52 + reward 4 + terminated 1 = 65; per env per launch the step
#       state (t 4, pos 4, cash 8) read + written 32 and the market position (ep 4, t 4,
#       S 8, C 4, P 4) read + written 48 = 80
LDS_STEP_B, LDS_STATE_B = 65, 80
# Tile kernels (he_step; he_rollout with a liability book or HE_LDS_ROLLOUT=0): the market
# is written to an HBM tile [M+1][N] by market_kernel and read back by the step kernel.
# Tile records per env-step:
#   "gbm"        12-B {S, C, P} + 12-B {greeks}   (GBM below GREEKS_IN_STEP_MIN_ENVS envs)
#   "gbm_step"   12-B {S, C, P} only              (GBM from there: the step kernel
#                                                  evaluates the f32 obs greeks itself)
#   "heston"     16-B {S, v, C, P} + 16-B {greeks, lag}
# he_step (step1_kernel): reads state 16 + action 8 + tile slots (pre A, post A, post B)
#   36 | 24 | 48; writes state 16 + obs 52 + reward 4 + terminated 1 + truncated 1
# he_rollout step_kernel (K steps): per step action 8 + tile post slots 24 | 12 | 32 + obs
#   52 + reward 4 + terminated 1; per launch state 32 + pre slot 12 | 12 | 16
GREEKS_IN_STEP_MIN_ENVS = 262144  # hedge_env.hip kGreeksInStepMinEnvs
STEP_BYTES_PER_ENV = {"gbm": 134, "gbm_step": 122, "heston": 146,
                      # replay he_step: state 16 + path 4 + S0 4 + action 8 + table rows (pre {S,v,C,P}
                      # 16, post 16, post greeks 16) + obs 52 + reward 4 + flags 2 + state written 16
                      "replay": 154}
# Replay rollouts (step_kernel, K fused steps): per env-step action 8 + the path row's
# {S, v, C, P} 16 and {greeks, lag} 16 + obs 52 + reward 4 + terminated 1; per launch the
# state (t, pos, cash) read + written 32, path + S0 read 8, the pre-step row 16.  SURVEY 8(d)
# prices replay at its generate-mode figure + the 16-B gather of S, v, C, P at t + 1.
REPLAY_ROLLOUT_B, REPLAY_STATE_B, SURVEY_REPLAY_GATHER_B = 97, 56, 16
# lds_replay_kernel: per env-step action 8 + the row's {S, v, C, P} 16 (its greeks are evaluated
# on chip) + obs 52 + reward 4 + terminated 1; per launch the state above + the episode sums
# (44 r+w) + the loaders' PCG64 words (40 r+w) and path / S0 written
LDS_REPLAY_STEP_B, LDS_REPLAY_STATE_B = 81, 56 + 88 + 80 + 8
ROLLOUT_BYTES_PER_ENV = {"gbm": 89, "gbm_step": 77, "heston": 97}
ROLLOUT_STATE_BYTES = {"gbm": 44, "gbm_step": 44, "heston": 48}
# market_kernel per env-step: tile records written; per env and block: the block-start
# state read (ep 4, t 4, S 8, C 4, P 4), written back to `cur` and to the rewind copy
# `bak` (3 x 24), + v (Heston) and the running max (book) at 8 B each, 3 times
MARKET_BYTES_PER_ENV = {"gbm": 24, "gbm_step": 12, "heston": 32}
MARKET_STATE_BYTES = 72


def lds_rollout(cfg):
    """he_rollout runs lds_rollout_kernel (GBM or Heston, with or without a book, unless
    HE_LDS_ROLLOUT=0)."""
    return cfg["mode"] in ("gbm", "heston") and os.environ.get("HE_LDS_ROLLOUT", "1") != "0"


def fused_market():
    return os.environ.get("HE_FUSED_MARKET", "1") != "0"


def tile_layout(mode, n):
    if mode in ("heston", "replay"):
        return mode
    thr = int(os.environ.get("HE_GREEKS_IN_STEP_MIN_ENVS") or GREEKS_IN_STEP_MIN_ENVS)
    return "gbm_step" if n >= thr else "gbm"


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# >= 2 episodes of 252 steps; 25,600 = 100 launches of the K = 256 rollout, so
# the timed region's per-launch device time averages over 100 dispatches (~30 ms at config 2:
# over 10 the same box read 292 and 318 us in two processes, r03s34)
MIN_TIMED_STEPS = 25600
M_BLOCK = 64           # market block (he_config.market_block)

TRAIN_KW = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002,
                slippage_bps=1.0)  # train_ppo_v2.py:74-80
GEN = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=252)

# liability books (extension, include/hedge_env.h he_book_option): short options on S0 = 496.48
BOOK8 = [dict(type=t, strike=k, expiry=e, quantity=q) for t, k, e, q in (
    ("call", 500.0, 63, -20.0), ("put", 480.0, 63, -15.0), ("call", 520.0, 126, -10.0), ("put", 500.0, 126, -25.0),
    ("call", 470.0, 189, -5.0), ("put", 530.0, 189, -5.0), ("call", 496.0, 252, -40.0), ("put", 450.0, 252, -30.0))]
BARRIER_BOOK = [dict(type="uo_call", strike=496.0, barrier=570.0, expiry=252, quantity=-50.0)]

# BASELINE.json configs (configs[0] is the CPU case = cpu_baseline below)
CONFIGS = {
    2: dict(envs=65536, mode="gbm", gen=GEN, kw=TRAIN_KW,
            workload="configs[1]: 65,536 parallel envs/GPU, European call (BS rolling-ATM marks), GBM, "
                     "v2 env, train_ppo_v2 reward"),
    3: dict(envs=1048576, mode="gbm", gen=GEN, kw=dict(TRAIN_KW, slippage_bps=5.0),
            workload="configs[2]: 1,048,576 parallel envs/GPU, European call, GBM, proportional costs "
                     "(5 bp slippage + $0.65 commission)"),
    4: dict(envs=524288, mode="gbm", gen=dict(GEN, book=BOOK8), kw=TRAIN_KW,
            workload="configs[3]: 524,288 envs/GPU (4M over 8 GPUs), GBM, liability book of 8 European "
                     "options per env marked every step"),
    5: dict(envs=131072, mode="heston",
            gen=dict(GEN, heston_kappa=2.0, heston_theta=0.029028, heston_xi=0.3, heston_rho=-0.7, book=BARRIER_BOOK),
            kw=TRAIN_KW,
            workload="configs[4]: Heston full-truncation Euler (rho=-0.7) + up-and-out barrier call book, "
                     "131,072 envs/GPU (1M over 8 GPUs)"),
    # the agents' own workload: train_ppo_v2.py:40 replays paths_rbergomi_options_100k.npz (100,000
    # paths x 253 columns, 405 MB as f32 {S, v, C, P}, past the 256 MB Infinity Cache) through
    # hedging_env_v2.py:223-231; a synthetic table of that shape in the reference NPZ layout
    6: dict(envs=65536, mode="replay", gen=GEN, kw=TRAIN_KW, table=dict(paths=100000, cols=253),
            workload="replay (train_ppo_v2.py:40): 65,536 envs/GPU replaying a synthetic 100,000 x 253 path table "
                     "in the reference NPZ layout (paths, volatilities, call/put_prices_atm), v2 env, "
                     "train_ppo_v2 reward"),
}

_TABLES = {}


def replay_tables(paths, cols, seed=2025):
    """A synthetic table in the reference NPZ layout (rbergomi_sim.py:528 keys, f32 as
    hedging_env_v2.py:36-41 loads them): S = a GBM-like path from S0 = 496.48 with a
    lognormal variance v, C / P = Black-Scholes rolling-ATM marks (30-day tenor, r = 0.04)
    at K = round(S_t) and sigma = sqrt(v_t), columns 0 .. cols - 2."""
    key = (paths, cols, seed)
    if key in _TABLES:
        return _TABLES[key]
    from scipy.special import ndtr
    rng = np.random.default_rng(seed)
    T = cols - 1
    dt, r, tenor = 1 / 252, 0.04, 30 / 252
    xi = 0.029028
    S = np.empty((paths, cols), np.float32)
    v = np.empty((paths, cols), np.float32)
    C = np.empty((paths, T), np.float32)
    P = np.empty((paths, T), np.float32)
    for a in range(0, paths, 12500):  # bounded f64 temporaries
        b = min(paths, a + 12500)
        m = b - a
        wv = np.cumsum(rng.standard_normal((m, cols)) * np.sqrt(dt), axis=1)
        vv = xi * np.exp(1.5 * wv - 0.5 * 1.5 ** 2 * np.arange(cols) * dt)
        z = rng.standard_normal((m, T))
        lr = (r - 0.5 * vv[:, :-1]) * dt + np.sqrt(vv[:, :-1] * dt) * z
        SS = 496.48 * np.exp(np.concatenate([np.zeros((m, 1)), np.cumsum(lr, axis=1)], axis=1))
        S[a:b], v[a:b] = SS, vv
        s, K, sig = SS[:, :-1], np.round(SS[:, :-1]), np.sqrt(vv[:, :-1])
        d1 = (np.log(s / K) + (r + 0.5 * sig * sig) * tenor) / (sig * np.sqrt(tenor))
        d2 = d1 - sig * np.sqrt(tenor)
        Kd = K * np.exp(-r * tenor)
        C[a:b] = s * ndtr(d1) - Kd * ndtr(d2)
        P[a:b] = Kd * ndtr(-d2) - s * ndtr(-d1)
    _TABLES[key] = (S, v, C, P)
    return _TABLES[key]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help=f"env: timed env-steps (default and floor {MIN_TIMED_STEPS}); rbergomi: launches (default 5)")
    ap.add_argument("--warmup", type=int, default=None, help="env: default 256; rbergomi: default 1")
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS), help="BASELINE.json config")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the config's)")
    ap.add_argument("--mode", choices=["rollout", "graph", "eager"], default="rollout")
    ap.add_argument("--rollout-k", type=int, default=None,
                    help="steps per he_rollout call (default: 256, the n_steps rollout-buffer boundary of "
                         "train_ppo_v2.py:48, on the LDS path; 64 on the tile path)")
    ap.add_argument("--no-step-api", action="store_true", help="skip the secondary graph-mode he_step run")
    ap.add_argument("--no-sb3-api", action="store_true", help="skip the host-API (SB3 VecEnv / single env) timing")
    ap.add_argument("--no-policy-api", action="store_true",
                    help="skip the closed-loop baseline-policy rollout (he_rollout_policy) timing")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="seconds per CPU-baseline leg (4 legs)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic pass")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launch-dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dist-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--action-sets", type=int, default=1,
                    help="rollout mode: cycle through this many distinct pre-generated action buffers (a "
                         "footprint past the 256 MB Infinity Cache; default 1)")
    ap.add_argument("--workload", choices=["env", "rbergomi"], default="env",
                    help="env: the hedging-env step (headline); rbergomi: the rough-Bergomi MC mark generator")
    ap.add_argument("--rb-paths", type=int, default=2048, help="rbergomi: paths per GPU (x 252 days x call/put)")
    ap.add_argument("--rb-normals", choices=["f64", "f32"], default="f64")
    ap.add_argument("--gather-rollout", action="store_true",
                    help="N > 1: also all-gather each boundary's rollout tensors (obs / reward / terminated of "
                         "the last he_rollout) in global env order (SURVEY 8(e): small N only)")
    args = ap.parse_args(argv)
    if args.workload == "env":
        args.steps = MIN_TIMED_STEPS if args.steps is None else args.steps
        args.warmup = 256 if args.warmup is None else args.warmup
    return args


def _cpu_sample(seconds, seed=42, barrier=None, n=256, offset=0):
    """One host core: the oracle (NumPy restatement of the reference env) on n envs
    (global env ids offset .. offset + n - 1 of the GBM workload)."""
    from oracle.hedging_oracle import OracleVecEnv
    env = OracleVecEnv(n, mode="gbm", gen=dict(GEN, seed=seed, env_offset=offset), **TRAIN_KW)
    env.seed_envs_at(np.arange(n), [seed] * n)
    env.reset()
    rng = np.random.default_rng(seed + offset)
    acts = rng.uniform(-1, 1, size=(8, n, 2)).astype(np.float32)
    for k in range(2):
        env.step(acts[k])
    if barrier is not None:
        barrier.wait()
    steps = 0
    t0 = time.perf_counter()
    while True:
        env.step(acts[steps % 8])
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return n * steps, el


_BARRIER = None


def _pool_init(b):
    global _BARRIER
    _BARRIER = b


def _pool_task(a):
    return _cpu_sample(a[0], a[1], _BARRIER, n=a[2], offset=a[3])


def _cpu_all_cores(seconds, procs, n_per, shard):
    """procs forked processes, one thread each, started together (a barrier)."""
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    b = ctx.Barrier(procs)
    with ctx.Pool(procs, initializer=_pool_init, initargs=(b,)) as pool:
        res = pool.map(_pool_task, [(seconds, 42 if shard else 42 + i, n_per, i * n_per if shard else 0)
                                    for i in range(procs)])
    return sum(s / e for s, e in res)


def host_cores():
    """(cores to use, affinity-mask count, where the first number comes from).

    SURVEY 8(d) asks for every host core in the affinity mask.  On the GPU pool the mask
    shows the whole machine (256 CPUs) while the job's share is the per-GPU grant the pool
    exports as OMP_NUM_THREADS (16 per GPU; the pool's rules: "size worker pools to the box's
    CPU share (16 for one GPU): nproc and os.cpu_count() show the whole machine's CPUs") --
    a pool of 256 workers would run on other jobs' cores.  So: the affinity count, capped by
    that grant when the environment states one."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    grant = os.environ.get("OMP_NUM_THREADS", "")
    if grant.isdigit() and 0 < int(grant) < avail:
        return int(grant), avail, (f"OMP_NUM_THREADS={grant}: the host cores this job is granted per GPU "
                                   f"({avail} CPUs in the affinity mask belong to the whole machine)")
    return avail, avail, f"every core of the affinity mask ({avail})"


def cpu_baseline(seconds):
    """SURVEY 8(d) / BASELINE.md section 2: the oracle on the host at N = 65,536 (the
    headline workload) and N = 256 (config 1), one process with one thread, then all
    granted cores (host_cores(): one process per core; at 65,536 each process steps its
    65,536 / P shard of the global env ids).  `value` is the 65,536-env all-cores rate.

    Must run before anything initialises the GPU: the all-core legs fork worker processes.
    """
    N = CONFIGS[2]["envs"]
    procs, avail, why = host_cores()
    s1, e1 = _cpu_sample(seconds, n=N)
    vN = _cpu_all_cores(seconds, procs, N // procs, shard=True)
    s256, e256 = _cpu_sample(seconds)
    v256 = _cpu_all_cores(seconds, procs, 256, shard=False)
    return dict(value=vN, unit="env-steps/s", cores=procs, affinity_cores=avail, cores_source=why, kind="port",
                sample=f"oracle/hedging_oracle.py OracleVecEnv GBM (the headline workload), {N} envs as {procs} "
                       f"processes x {N // procs} envs x {seconds:.0f} s (NumPy, 1 thread each; {avail} cores in "
                       f"affinity mask)",
                single_core_value=s1 / e1,
                single_core_sample=f"{N} envs x {s1 // N} steps in one process ({e1:.1f} s, 1 thread)",
                n256_value=v256,
                n256_sample=f"256 envs per process, {procs} processes x {seconds:.0f} s (BASELINE config 1)",
                n256_single_core_value=s256 / e256,
                n256_single_core_sample=f"256 envs x {s256 // 256} steps ({e256:.1f} s, 1 thread)",
                **REFERENCE_CPU)


# The reference's own env (hedging_env_v2.py, unmodified, record_metrics=True) on 256 envs,
# measured in the build container (8-core Xeon, nproc = 8), not on the GPU box:
# SURVEY.md section 6 / BASELINE.md:18-20
REFERENCE_CPU = dict(
    reference_value=4782.0, reference_value_8proc=31904.0,
    reference_sample="container measurement (build container, nproc=8, not the GPU box): the reference's "
                     "hedging_env_v2.py, 256 envs, serial DummyVecEnv-style loop = 4,782 env-steps/s on 1 process; "
                     "8 fork processes x 32 envs = 31,904 env-steps/s (SURVEY.md section 6, BASELINE.md:18-20)")


def make_env(args, dev, rank=0, prefetch="auto", offset=None):
    """The config's env handle of args.envs envs at global env ids offset .. (default rank's)."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    cfg = CONFIGS[args.config]
    off = rank * args.envs if offset is None else offset
    if cfg["mode"] == "replay":
        # env i of rank r draws its episodes from PCG64(SeedSequence(seed + r * envs + i)),
        # the reference's per-env reset(seed) streams (hedging_env_v2.py:146-150)
        env = HedgingVecEnv(args.envs, tables=replay_tables(**cfg["table"]), seed=args.seed,
                            global_env_offset=off, device=dev, return_numpy=False, info_keys=(),
                            **cfg["kw"])
        env.reset_tensors()
        return env
    env = HedgingVecEnv(args.envs, mode=cfg["mode"], generate=cfg["gen"], seed=args.seed,
                        global_env_offset=off, device=dev, return_numpy=False, info_keys=(),
                        market_prefetch=prefetch, **cfg["kw"])
    env.reset_tensors()
    return env


def bench_actions(n, rank, dev, sets=1):
    """The pre-generated U(-1, 1) actions [256, n, 2] of rank `rank` (seed 1234 + rank).
    sets > 1 (--action-sets): [sets, 256, n, 2], set s from seed 1234 + rank + 7919 s, the
    rollouts cycling through them (a footprint past the 256 MB Infinity Cache: DESIGN 9)."""
    if sets > 1:
        return torch.stack([bench_actions(n, rank + 7919 * s, dev) for s in range(sets)])
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    return torch.rand((256, n, 2), device=dev, generator=g) * 2 - 1


# ---------------------------------------------------------------------- shard check
# After the timed region each rank re-runs its NEIGHBOUR's shard (rank (r + 1) % world) in a
# handle of its own of the same size, with the neighbour's actions and the same launches, and
# compares the bits of its episode summaries with the rows the all-gather delivered: the shards
# are a partition of one global env set whatever the GPU count (Philox keyed by the global env
# id), and the gather puts them in global env order.  At one rank it checks the
# handle's own envs.  The whole shard, not a slice: the check's launches then have the timed
# launches' grid, so a rocprofv3 --stats summary of the run averages one launch shape (a 64-env
# slice ran 1-workgroup launches of the same kernel that pulled the average down).
SHARD_CHECK_ENVS = None   # None: the whole shard


def shard_check_slice(rank, world, n, m=SHARD_CHECK_ENVS):
    """(neighbour rank, its first checked env, count): the last min(m, n) envs of (r + 1) % world
    (m None: all n)."""
    m = n if m is None else min(m, n)
    return (rank + 1) % world, n - m, m


def shard_check_verdict(dist, got, gathered, nb, j0, n, device="cpu"):
    """Bits of `got` [m, 4] against rows nb * n + j0 .. of `gathered` [world * n, 4]; every rank's
    result combined (MIN over ranks) -> the line's `shard_check`."""
    m = int(got.shape[0])
    ref = gathered[nb * n + j0: nb * n + j0 + m]
    a = got.detach().cpu().contiguous().view(torch.int32)
    b = ref.detach().cpu().contiguous().view(torch.int32)
    same = a.shape == b.shape and bool(torch.equal(a, b))
    bad_rows = 0 if same else int((a != b).any(dim=1).sum()) if a.shape == b.shape else m
    ok = torch.tensor([1 if same else 0], dtype=torch.int64, device=device)
    bad = torch.tensor([bad_rows], dtype=torch.int64, device=device)
    if dist is not None:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        dist.all_reduce(bad, op=dist.ReduceOp.SUM)
    world = dist.get_world_size() if dist is not None else 1
    all_ok = bool(int(ok.item()))
    finished = int((ref[:, 3] > 0).sum().item()) if m else 0
    return dict(result="bit-identical" if all_ok else "MISMATCH", envs_per_rank=m, ranks=world,
                mismatched_rows=int(bad.item()), finished_episodes_in_checked_rows=finished,
                what="each rank re-ran the last %d envs of rank (r + 1) %% world in a %d-env handle at their global "
                     "env ids (the neighbour's actions, the same launches) and compared the bits of their "
                     "he_episode_summaries with the all-gathered rows" % (m, m))


def shard_check_run(args, dev, stream, runs, nb, j0, m):
    """The checked envs' episode summaries [m, 4]: a handle of m envs at global ids nb * n + j0 ..,
    driven by the same sequence of Runner.run() calls `runs` with rank nb's actions."""
    import copy
    a2 = copy.copy(args)
    a2.envs = m
    acts = bench_actions(args.envs, nb, dev, args.action_sets)[..., j0:j0 + m, :].contiguous()
    env = make_env(a2, dev, offset=nb * args.envs + j0)
    r = Runner(a2, env, "rollout", acts, stream)
    with torch.cuda.stream(stream):
        for k in runs:
            r.run(k)
        out = env.episode_summaries()
    torch.cuda.synchronize()
    env.close()
    return out


class Runner:
    """Enqueues env-steps of one handle in one mode (rollout / graph / eager)."""

    def __init__(self, args, env, mode, acts, stream, dist=None, gathered=None):
        # acts [256, n, 2], or [S, 256, n, 2] (--action-sets S): launch i reads set i % S
        self.sets = acts if acts.dim() == 4 else acts.unsqueeze(0)
        self.launches = 0
        acts = self.sets[0]
        self.args, self.env, self.mode, self.acts, self.stream = args, env, mode, acts, stream
        self.dist, self.gathered = dist, gathered
        self.summaries = torch.zeros((args.envs, 4), dtype=torch.float32, device=acts.device)
        self.gathers = 0
        self.boundary_events = []   # (start, summaries+gather done, rollout tensors gathered) per boundary
        self.rollout_gathered = None
        self.lib, self.h = env.lib, env._h
        self.ring = acts.shape[0]
        n = args.envs
        dev = acts.device
        self.chunk = args.rollout_k if mode == "rollout" else (M_BLOCK if mode == "graph" else 1)
        if mode == "rollout":
            RK = args.rollout_k
            self.ro = torch.empty((RK, n, 13), dtype=torch.float32, device=dev)
            self.rr = torch.empty((RK, n), dtype=torch.float32, device=dev)
            self.rt = torch.empty((RK, n), dtype=torch.uint8, device=dev)
        self.graphs = []
        self.replays = 0
        self.runs = []
        if mode == "graph":
            with torch.cuda.stream(stream):
                # one eager block first, so each captured graph is the steady state
                # [fork: market_kernel(b+1) on the side stream || 64 x step1_kernel(b)] + join
                for j in range(M_BLOCK):
                    self.step(j, stream.cuda_stream)
                env.sync_market()
                torch.cuda.synchronize()
                for gi in range(self.ring // M_BLOCK):
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=stream):
                        cs = torch.cuda.current_stream().cuda_stream
                        for j in range(M_BLOCK):
                            self.step(gi * M_BLOCK + j, cs)
                        env.sync_market()
                    self.graphs.append(gr)
            torch.cuda.synchronize()

    def step(self, k, s):
        e = self.env
        st = self.lib.he_step(self.h, self.acts[k % self.ring].data_ptr(), e._obs.data_ptr(), e._rew.data_ptr(),
                              e._term.data_ptr(), e._trunc.data_ptr(), e._tobs.data_ptr(), None, s)
        if st:
            raise RuntimeError(self.lib.he_last_error(self.h).decode())

    def rollout(self, done, s):
        RK = self.args.rollout_k
        a0 = done % self.ring
        acts = self.sets[self.launches % self.sets.shape[0]]
        self.launches += 1
        a = acts[a0:a0 + RK] if a0 + RK <= self.ring else acts[:RK]
        st = self.lib.he_rollout(self.h, RK, a.data_ptr(), self.ro.data_ptr(), self.rr.data_ptr(),
                                 self.rt.data_ptr(), s)
        if st:
            raise RuntimeError(self.lib.he_last_error(self.h).decode())

    def run(self, steps):
        """Enqueue `steps` env-steps (a multiple of the chunk) on self.stream."""
        self.runs.append(steps)   # the call sequence, replayed by the shard check
        done = 0
        cs = self.stream.cuda_stream
        while done < steps:
            if self.mode == "graph":
                self.graphs[self.replays % len(self.graphs)].replay()
                self.replays += 1
            elif self.mode == "eager":
                self.step(done, cs)
            else:
                self.rollout(done, cs)
            done += self.chunk
            if self.dist is not None and done % GATHER_EVERY == 0:
                self.gather(cs)

    def gather(self, cs):
        """The rollout-buffer boundary (train_ppo_v2.py:48, n_steps = 256): every rank's
        per-env episode summaries, stream-ordered behind the rollouts that made them; with
        --gather-rollout also the last rollout's obs / reward / terminated tensors
        [K, N, ...] of every rank, in global env order ([K, world * N, ...]).  Each boundary
        is bracketed by events on the launching stream (RCCL: the collective's completion
        is ordered into this stream; gloo: the host copy syncs it)."""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(self.stream)
        st = self.lib.he_episode_summaries(self.h, self.summaries.data_ptr(), cs)
        if st:
            raise RuntimeError(self.lib.he_last_error(self.h).decode())
        gather_summaries(self.dist, self.summaries, self.gathered)
        ev[1].record(self.stream)
        if self.args.gather_rollout and self.mode == "rollout":
            from cantorrl_amd import dist as hd
            host = self.dist.get_backend() == "gloo"
            self.rollout_gathered = [hd.gather_rollout(t.cpu() if host else t, env_dim=1)
                                     for t in (self.ro, self.rr, self.rt)]
        ev[2].record(self.stream)
        self.boundary_events.append(ev)
        self.gathers += 1

    def boundary_us(self):
        """Mean device time per boundary on the stream: (summaries + gather, rollout-tensor
        gather) in us, over the timed region's boundaries."""
        if not self.boundary_events:
            return None, None
        a = np.array([e[0].elapsed_time(e[1]) for e in self.boundary_events]) * 1e3
        b = np.array([e[1].elapsed_time(e[2]) for e in self.boundary_events]) * 1e3
        return float(a.mean()), (float(b.mean()) if self.args.gather_rollout else None)


GATHER_EVERY = 256  # train_ppo_v2.py:48 n_steps
# Fail fast: a rank that never joins, or a collective that stalls, ends the
# run after this many seconds (init_process_group's timeout) instead of the driver's wall limit
DIST_TIMEOUT_S = float(os.environ.get("BENCH_DIST_TIMEOUT", "120"))
# the `--gpus N` launcher's wall limit on its torch.distributed.run child
LAUNCH_TIMEOUT_S = float(os.environ.get("BENCH_LAUNCH_TIMEOUT", "900"))


def rank_phase(phase, rank=None, world=None):
    """One rank's progress record: a line on stderr ("[bench rank r/w] phase (t s)") and, under
    the `--gpus N` launcher, the rank's status file, which the launcher reads to name the ranks
    that did not finish when the child fails or times out."""
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    if world <= 1:
        return
    t = round(time.time() - _T0, 2)
    print(f"[bench rank {rank}/{world}] {phase} ({t} s)", file=sys.stderr, flush=True)
    d = os.environ.get("BENCH_RANK_STATUS_DIR")
    if d and os.path.isdir(d):
        with open(os.path.join(d, f"rank{rank}"), "a") as fh:
            fh.write(f"{t} {phase}\n")


_T0 = time.time()


def init_dist(local):
    """One rank per GPU over RCCL (backend "nccl").  BENCH_DIST_BACKEND=gloo is the
    rehearsal of the N-rank path on a box with fewer GPUs than ranks (ranks share
    device local % device_count, host-side collectives; on a host with no GPU, the CPU
    test of the launcher); the driver's runs use RCCL.  The process group's timeout is
    DIST_TIMEOUT_S: a rank that never joins fails the others' init within it."""
    import datetime
    import torch.distributed as dist
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    timeout = datetime.timedelta(seconds=DIST_TIMEOUT_S)
    rank_phase("init_process_group(%s, timeout %g s)" % (backend, DIST_TIMEOUT_S))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    else:
        if torch.cuda.is_available():
            torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dist.init_process_group(backend, timeout=timeout)
    rank_phase("ready")
    return dist, backend


def dist_selftest():
    """`--dist-selftest` (tests/test_bench_launcher_cpu.py): the ranks' rendezvous and one
    collective only, through the real launcher path.  BENCH_TEST_STALL_RANK=r makes rank r
    never join (it sleeps), to show the run fails within DIST_TIMEOUT_S and names it."""
    stall = os.environ.get("BENCH_TEST_STALL_RANK")
    rank = int(os.environ.get("RANK", "0"))
    rank_phase("start")
    if stall is not None and int(stall) == rank:
        rank_phase("stalling (BENCH_TEST_STALL_RANK)")
        time.sleep(3600)
    dist, _ = init_dist(int(os.environ.get("LOCAL_RANK", "0")))
    t = torch.ones(1)
    dist.all_reduce(t)
    rank_phase("all_reduce %g" % float(t.item()))
    dist.destroy_process_group()
    rank_phase("done")


def gather_summaries(dist, local, gathered):
    """All-gather the per-env episode summaries [n, 4] {return, sum P&L, sum cost, length}
    of every rank into gathered [world * n, 4], rank-major: row r * n + i is global env
    r * n + i (env ids are offset by rank, so this is the single-process [world * n, 4]).
    RCCL (device tensors, on the current stream) or gloo (host tensors)."""
    if gathered.is_cuda:
        dist.all_gather_into_tensor(gathered, local)
    else:
        dist.all_gather(list(gathered.chunk(dist.get_world_size())), local.to(gathered.device))
    return gathered


def summarize_payload(gathered):
    """The gathered payload in a few numbers (the Monitor-style episode stats the
    reference logs at the boundary, train_ppo_v2.py:119)."""
    g = gathered.double().cpu()
    fin = g[:, 3] > 0
    nf = int(fin.sum())
    out = dict(envs=int(g.shape[0]), envs_with_finished_episode=nf)
    if nf:
        out.update(mean_return=float(g[fin, 0].mean()), mean_pnl=float(g[fin, 1].mean()),
                   mean_cost=float(g[fin, 2].mean()), mean_length=float(g[fin, 3].mean()))
    return out


def probe(args):
    """Short run for counter collection (the headline mode's kernel)."""
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    env = make_env(args, dev)
    acts = torch.rand((256, args.envs, 2), device=dev) * 2 - 1
    stream = torch.cuda.Stream(device=dev)
    r = Runner(args, env, "eager" if args.mode == "graph" else args.mode, acts, stream)
    with torch.cuda.stream(stream):
        r.run(r.chunk * (8 if args.mode == "rollout" else 128))
    torch.cuda.synchronize()
    env.close()


STEP_KERNELS = r"step1?_kernel|step_market_kernel|lds_rollout_kernel|lds_replay_kernel"


def pmc_pass(args, counters, kernels=STEP_KERNELS, probe_argv=None):
    """One rocprofv3 --pmc pass of `bench.py --probe` (a child process: this one has not
    touched the GPU) -> {kernel short name: {counter: mean per dispatch}} for the
    kernels matching `kernels` (the first dispatches of each skipped: warm-up).
    `probe_argv`: the probe's own arguments (default: the env workload of `args`)."""
    import csv
    import glob
    import re
    import shutil
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    if probe_argv is None:
        probe_argv = ["--envs", str(args.envs), "--config", str(args.config), "--mode", args.mode,
                      "--rollout-k", str(args.rollout_k)]
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", td, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--probe", *probe_argv]
        try:
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=240, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
        except Exception as e:  # noqa: BLE001
            return None, f"rocprofv3 --pmc {' '.join(counters)} failed: {e}"
        rows = {}
        for fn in glob.glob(os.path.join(td, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as fh:
                for r in csv.DictReader(fh):
                    m = re.search(kernels, r.get("Kernel_Name", ""))
                    if m and r.get("Counter_Name") in counters:
                        k = m.group(0)
                        rows.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if not rows:
        return None, f"no {counters} rows for {kernels}"
    skip = 2 if args.mode == "rollout" else 8
    return {k: {c: float(np.mean(v[skip:] if len(v) > 2 * skip else v)) for c, v in d.items()}
            for k, d in rows.items()}, None


READ_REQ_COUNTERS = ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"]


def traffic_bytes(c):
    """HBM bytes from one kernel's counters {name: per-dispatch value}: the L2's memory-side read
    requests by size (gfx950's TCC_EA0_RDREQ_{32B,64B,128B}; any request in none of the three
    counted at 64 B) + WRITE_SIZE (KiB).  Calibrated on known byte counts (tools/traffic_calib.py,
    profiles/r05s10_traffic_calib.log): a 1 GiB read as a coalesced stream, as 64-B half lines
    from two waves and as a 128-B line per lane each gives 1,073.8 MB = its bytes, where
    FETCH_SIZE gives half (MI355X_MICROARCH.md "HBM": rocprofv3's gfx950 FETCH_SIZE takes
    TCC_BUBBLE for the 128-B requests)."""
    r32, r64, r128 = (c["TCC_EA0_RDREQ_%s_sum" % w] for w in ("32B", "64B", "128B"))
    other = max(c["TCC_EA0_RDREQ_sum"] - r32 - r64 - r128, 0.0)
    return 32.0 * r32 + 64.0 * (r64 + other) + 128.0 * r128 + 1024.0 * c["WRITE_SIZE"]


def pmc_traffic(args, kernels=STEP_KERNELS, probe_argv=None):
    """HBM bytes per step-kernel launch from rocprofv3 PMC counters (traffic_bytes): the sized
    read requests in one pass, WRITE_SIZE in another.  Runs BEFORE this process touches the
    GPU; the profiled program is a child (`rocprofv3 ... -- python3`)."""
    vals = {}
    for ctrs in (READ_REQ_COUNTERS, ["WRITE_SIZE"]):
        res, err = pmc_pass(args, ctrs, kernels, probe_argv)
        if res is None:
            return None, err
        for ctr in ctrs:
            vals[ctr] = sum(d[ctr] for d in res.values() if ctr in d)
    return traffic_bytes(vals), vals


VALU_COUNTERS = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                 "SQ_INSTS_VALU_TRANS_F64", "GRBM_GUI_ACTIVE"]
FP64_VECTOR_PEAK_TFLOPS = 78.6  # half the 157.3 TF f32 vector rate (MI355X_MICROARCH.md): f64 FMA issues at 1/2


def pmc_valu(args):
    """The VALU side of the step and market kernels (one --pmc pass): per dispatch, wave
    instructions per SIMD-cycle (cycles = GRBM_GUI_ACTIVE / 8, the guide's per-XCD sum)
    against the issue bound of the kernel's f64 / other mix (a wave64 VALU instruction
    every 2 cycles per SIMD, f64 every 4), and the f64 FLOP count per dispatch."""
    res, err = pmc_pass(args, VALU_COUNTERS, STEP_KERNELS + "|market_kernel")
    if res is None:
        return None, err
    return valu_summary(res), None


def valu_summary(res):
    """{kernel: {counter: mean per dispatch}} of a VALU_COUNTERS pass -> per kernel the issue
    rate, its bound for the kernel's f64 share and the f64 FLOP per dispatch."""
    out = {}
    for k, d in res.items():
        if "SQ_INSTS_VALU" not in d or not d.get("GRBM_GUI_ACTIVE"):
            continue
        f64 = sum(d.get(c, 0.0) for c in VALU_COUNTERS[1:5])
        share = f64 / d["SQ_INSTS_VALU"] if d["SQ_INSTS_VALU"] else 0.0
        cycles = d["GRBM_GUI_ACTIVE"] / 8.0
        issue = d["SQ_INSTS_VALU"] / (cycles * 1024.0)
        bound = 1.0 / (2.0 * (1.0 - share) + 4.0 * share)
        out[k] = dict(valu_insts=d["SQ_INSTS_VALU"], f64_share=round(share, 4),
                      issue_per_simd_cycle=round(issue, 4), issue_bound_per_simd_cycle=round(bound, 4),
                      valu_issue_frac=round(issue / bound, 4),
                      f64_flop=64.0 * (2.0 * d.get("SQ_INSTS_VALU_FMA_F64", 0.0) + d.get("SQ_INSTS_VALU_ADD_F64", 0.0)
                                       + d.get("SQ_INSTS_VALU_MUL_F64", 0.0)),
                      cycles_profiled=cycles)
    return out


class HipEvents:
    """hipEvent_t pairs from the HIP runtime torch (and libhedgeenv) use."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so.7")

    def create(self):
        e = ctypes.c_void_p()
        if self.hip.hipEventCreate(ctypes.byref(e)) != 0:
            raise RuntimeError("hipEventCreate failed")
        return e

    def record(self, e, stream):
        self.hip.hipEventRecord(e, ctypes.c_void_p(stream.cuda_stream))

    def elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        if self.hip.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def destroy(self, *evs):
        for e in evs:
            self.hip.hipEventDestroy(e)


def kernel_time_ms(hev, runner, nprobe):
    """Live duration of the step kernel: he_time_next_step brackets exactly the next
    step-kernel dispatch with HIP events on `runner.stream` (hipExtLaunchKernelGGL)."""
    env, lib, h, stream = runner.env, runner.lib, runner.h, runner.stream
    kev = [(hev.create(), hev.create()) for _ in range(nprobe)]
    env.reset_tensors()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for k in range(nprobe):
            lib.he_time_next_step(h, kev[k][0], kev[k][1])
            if runner.mode == "rollout":
                runner.rollout(k * runner.chunk, stream.cuda_stream)
            else:
                runner.step(k, stream.cuda_stream)
    torch.cuda.synchronize()
    kd = np.array([hev.elapsed_ms(a, b) for a, b in kev])
    for a, b in kev:
        hev.destroy(a, b)
    skip = 4 if runner.mode == "rollout" else 8
    return float(np.mean(kd[skip:]))


def market_time_ms(hev, args, dev, acts, stream):
    """market_kernel duration per block of M_BLOCK steps: he_step on a handle without
    prefetch, where it runs inside the he_step call of every block boundary."""
    env2 = make_env(args, dev, prefetch=False)
    m = []
    with torch.cuda.stream(stream):
        for k in range(4 * M_BLOCK):
            a, b = hev.create(), hev.create()
            hev.record(a, stream)
            st = env2.lib.he_step(env2._h, acts[k % acts.shape[0]].data_ptr(), env2._obs.data_ptr(),
                                  env2._rew.data_ptr(), env2._term.data_ptr(), env2._trunc.data_ptr(), None,
                                  None, stream.cuda_stream)
            hev.record(b, stream)
            if st:
                raise RuntimeError(env2.lib.he_last_error(env2._h).decode())
            m.append((a, b))
    torch.cuda.synchronize()
    d2 = np.array([hev.elapsed_ms(a, b) for a, b in m])
    for a, b in m:
        hev.destroy(a, b)
    env2.close()
    return float(np.median(d2[M_BLOCK::M_BLOCK])) - float(np.median(np.delete(d2, np.arange(0, 4 * M_BLOCK, M_BLOCK))))


# The GPU's clocks ramp up under sustained load: back-to-back 65,536-env launches measured
# 395-404 us each in the first ~10 ms after idle and 320 us from ~30 ms on
# (tools/launch_timing.py, r03s2).  The warm-up therefore runs for at least this long
# (whole chunks; the line reports the warm-up steps actually run beside the requested ones).
MIN_WARMUP_SECONDS = 0.5


def timed(runner, K, W, dist):
    """W untimed warm-up steps (extended to MIN_WARMUP_SECONDS of work; the count run is left
    in runner.warmup_steps), then exactly K timed steps between barriers; returns
    (max-over-ranks wall seconds, device ms on the stream)."""
    stream = runner.stream
    t_w = time.perf_counter()
    d_saved, runner.dist = runner.dist, None  # no gathers while warming: ranks' counts may differ
    with torch.cuda.stream(stream):
        runner.run(W)
    torch.cuda.synchronize()
    while time.perf_counter() - t_w < MIN_WARMUP_SECONDS:
        with torch.cuda.stream(stream):
            runner.run(runner.chunk * 4)
        torch.cuda.synchronize()
        W += runner.chunk * 4
    if dist is not None:  # every rank warms for the longest rank's count of steps
        w = torch.tensor([W], dtype=torch.int64,
                         device="cpu" if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        if int(w.item()) > W:
            with torch.cuda.stream(stream):
                runner.run(int(w.item()) - W)
            torch.cuda.synchronize()
            W = int(w.item())
    runner.dist = d_saved
    runner.boundary_events = []   # the timed region's boundaries only
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        runner.run(K)
        ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    runner.warmup_steps = W
    host = dist is not None and dist.get_backend() == "gloo"
    t = torch.tensor([wall], dtype=torch.float64,
                     device="cpu" if host else torch.device("cuda", torch.cuda.current_device()))
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), ev0.elapsed_time(ev1)


def roofline(mode, n, kern_ms, rk, book=False, market="gbm", lds=False):
    """The dominant kernel's roofline.  `achieved` = SURVEY 8(d)'s algorithmic bytes per
    launch / the kernel's average duration.  `kernel_bytes_per_launch` is what this
    kernel itself must move (the 8(d) I/O plus the market position; the tile kernels add
    their HBM market tile, reported apart as `overhead_bytes_per_launch`)."""
    overhead = 0
    if mode == "rollout":
        survey = n * (rk * SURVEY_ROLLOUT_B + SURVEY_ROLLOUT_STATE_B)
        if market == "replay":
            survey = n * (rk * (SURVEY_ROLLOUT_B + SURVEY_REPLAY_GATHER_B) + SURVEY_ROLLOUT_STATE_B)
            own = n * (rk * REPLAY_ROLLOUT_B + REPLAY_STATE_B)
            if os.environ.get("HE_LDS_ROLLOUT", "1") != "0":
                own = n * (rk * LDS_REPLAY_STEP_B + LDS_REPLAY_STATE_B)
                kname = ("lds_replay_kernel (he_rollout, replay, K=%d fused steps; a loader wave stages each "
                         "env's path rows in LDS one block ahead of the steppers)" % rk)
            else:
                kname = ("step_kernel (he_rollout, replay, K=%d fused steps; each env gathers its path row from "
                         "the table)" % rk)
        elif lds:
            # + the book's running max, + Heston's f64 variance (each read + written)
            own = n * (rk * LDS_STEP_B + LDS_STATE_B + (16 if book else 0) + (16 if market == "heston" else 0))
            kname = ("lds_rollout_kernel (he_rollout, K=%d fused steps; the market made in LDS by "
                     "producer waves, never written to HBM)" % rk)
        else:
            own = n * (rk * (65 + (8 if book else 0)) + 32)
            overhead = n * rk * (ROLLOUT_BYTES_PER_ENV[market] - 65) + n * (ROLLOUT_STATE_BYTES[market] - 32)
            kname = "step_kernel (he_rollout, K=%d fused steps, market tile in HBM)" % rk
            if fused_market() and not book:
                mstate = MARKET_STATE_BYTES + (24 if market == "heston" else 0)
                overhead += n * (rk * MARKET_BYTES_PER_ENV[market] + mstate)
                kname = ("step_market_kernel (he_rollout, K=%d fused steps + the next block's market "
                         "tile in the same grid)" % rk)
    else:
        survey = n * (SURVEY_STEP_B + (SURVEY_REPLAY_GATHER_B if market == "replay" else 0))
        own = n * (STEP_BYTES_PER_ENV[market] + (16 if book else 0))
        kname = "step1_kernel (he_step, K=1)"
    achieved = survey / (kern_ms * 1e-3) / 1e9
    return dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None, kernel=kname,
                kernel_us=round(kern_ms * 1e3, 3), bytes_model="SURVEY.md 8(d)", bytes_per_launch=int(survey),
                kernel_bytes_per_launch=int(own), overhead_bytes_per_launch=int(overhead),
                kernel_gbs=round(own / (kern_ms * 1e-3) / 1e9, 1))


def step_api_line(n, steps, wall, rf, pmc, layout):
    """The Gym-API (graph-mode he_step) sub-line.  Two fractions of 8 TB/s, both from the same
    kernel time: `frac` on the bytes step1_kernel itself must move (STEP_BYTES_PER_ENV[layout]:
    122 B per env when it evaluates the obs greeks, 134 B when it reads them from the market
    tile) and `frac_survey_8d` on SURVEY 8(d)'s 186 B per env-step (66 of step I/O + the 120-B
    state model, larger than this kernel's 16-B state) -- only the first is the kernel's own
    roofline.  `traffic` is the kernel's PMC HBM bytes per launch (traffic_bytes)."""
    kb = rf["kernel_bytes_per_launch"]
    kgbs = kb / (rf["kernel_us"] * 1e-6) / 1e9
    out = dict(mode="graph (he_step, one launch per step)", value=round(n * steps / wall, 1),
               ms_per_step=round(wall * 1e3 / steps, 6), kernel=rf["kernel"], kernel_us=rf["kernel_us"],
               kernel_bytes_per_launch=int(kb), kernel_bytes_per_env=int(kb // n), kernel_bytes_layout=layout,
               achieved_gbs=round(kgbs, 1), frac=round(kgbs / HBM_PEAK_GBS, 4),
               bytes_per_launch=rf["bytes_per_launch"], achieved_gbs_survey_8d=rf["achieved"],
               frac_survey_8d=rf["frac"], traffic=None)
    if pmc[0] is not None:
        out["traffic"] = int(pmc[0])
        out["traffic_over_kernel_bytes"] = round(pmc[0] / kb, 4)
        out["traffic_counters"] = {k: round(v, 1) for k, v in pmc[1].items()}
    else:
        out["traffic_note"] = pmc[1]
    return out


def config_bound(cfg):
    """The resource that bounds a configuration's dominant kernel, fixed per config (not by
    whether the counters ran): with a liability book or Heston the producers' f64 market work
    (8 Black-Scholes prices per env-step, the variance chain + barrier pricer) bounds the LDS
    kernel -- VALU issue; otherwise the step I/O -- HBM."""
    return "valu" if (cfg["gen"].get("book") or cfg["mode"] == "heston") else "hbm"


def finish_roofline(roof, cfg, valu, pmc, kern_ms):
    """Attach the PMC results (VALU issue, HBM traffic) to the HBM roofline `roof` and, for a
    VALU-bound configuration (config_bound), make the VALU issue rate the headline figure: the
    issue rate against the bound of the kernel's own f64 / other mix (a wave64 instruction
    every 2 cycles per SIMD, f64 every 4), the HBM side kept under "hbm".  Without the VALU
    pass such a line still says "valu" and leaves the figure null, with a note."""
    if valu[0]:
        # the dominant kernel by profiled cycles
        dom = max(valu[0], key=lambda k: valu[0][k]["cycles_profiled"])
        v = dict(valu[0][dom])
        if dom in ("lds_rollout_kernel", "lds_replay_kernel") or (dom.startswith("step") and "market" not in dom):
            v["f64_tflops"] = round(v["f64_flop"] / (kern_ms * 1e-3) / 1e12, 3)
            v["f64_frac_of_vector_peak"] = round(v["f64_tflops"] / FP64_VECTOR_PEAK_TFLOPS, 4)
        roof["valu"] = dict(kernel=dom, peak_f64_tflops=FP64_VECTOR_PEAK_TFLOPS, **v)
        roof["valu_by_kernel"] = valu[0]
    elif valu[1] != "skipped":
        roof["valu_note"] = valu[1]
    if pmc[0] is not None:
        roof["traffic"] = int(pmc[0])
        roof["traffic_over_bytes"] = round(pmc[0] / roof["bytes_per_launch"], 4)
        roof["traffic_counters"] = {k: round(v, 1) for k, v in pmc[1].items()}
    else:
        roof["traffic_note"] = pmc[1]
    if config_bound(cfg) != "valu":
        return roof
    hbm = {k: roof.pop(k) for k in ("achieved", "peak", "unit", "frac")}
    hbm["bound_note"] = "not the bound of this configuration (see valu)"
    v = roof.get("valu")
    if v is not None and v["kernel"] == "lds_rollout_kernel":
        head = dict(achieved=v["issue_per_simd_cycle"], peak=v["issue_bound_per_simd_cycle"], frac=v["valu_issue_frac"])
    else:
        head = dict(achieved=None, peak=None, frac=None)
        roof["valu_note"] = ("VALU issue not measured in this run (the PMC pass was %s): the bound is still VALU issue "
                             "of the LDS producers; see the HBM figure under 'hbm' for the I/O side" %
                             (valu[1] if valu[1] else "absent"))
    return dict(bound="valu", unit="VALU wave-instructions per SIMD-cycle", traffic=roof.pop("traffic", None),
                hbm=hbm, **head, **{k: x for k, x in roof.items() if k != "bound"})


# ---------------------------------------------------------------------- the host (SB3 / gym) API
# The reference's own single env stepped in a serial loop, measured in the build container
# (SURVEY.md section 6 / BASELINE.md:18-20: 4,782 env-steps/s over 256 envs on one core,
# ~209 us per HedgingEnv.step) -- what `baselines.py:45-51` and `delta_and_nothing.py:69-88`
# drive today.
REFERENCE_SINGLE_ENV_STEPS_S = 4782.0
SB3_API_ENVS = (2, 256, 65536)   # N_ENVS = 2 (train_ppo_v2.py:45), BASELINE config 1, the headline
# the 9 info keys of the reference's evaluation loop (train_ppo_v2.py:482-499)
EVAL_INFO_KEYS = ("per_share_step_pnl", "transaction_costs_total", "scaled_float_call", "scaled_float_put",
                  "requested_calls_rounded_clipped", "requested_puts_rounded_clipped", "actual_calls_traded",
                  "actual_puts_traded", "raw_pnl_deviation_abs")


def sb3_collect_pass(infos, dones, ep_info_buffer):
    """What SB3 2.6.0's collect_rollouts does with a step's infos on the host (restated: SB3 is not
    installed): _update_info_buffer -- info.get("episode") / info.get("is_success") of EVERY row --
    and the truncation-bootstrap loop over the done rows (on_policy_algorithm.py)."""
    for idx, info in enumerate(infos):
        maybe_ep_info = info.get("episode")
        maybe_is_success = info.get("is_success")
        if maybe_ep_info is not None:
            ep_info_buffer.extend([maybe_ep_info])
        if maybe_is_success is not None and dones[idx]:
            pass
    for idx, done in enumerate(dones):
        if done and infos[idx].get("terminal_observation") is not None and infos[idx].get("TimeLimit.truncated", False):
            pass


def eval_pass(infos, n, sums):
    """The info reads of train_ppo_v2.py:481-499 per env per step (9 keys; the caller's own
    action-log dict is the same work on either side of the swap and is left out)."""
    for i in range(n):
        sums[0] += infos[i].get('per_share_step_pnl', 0.0)
        sums[1] += infos[i].get('transaction_costs_total', 0.0)
        sums[2] += float(infos[i].get('scaled_float_call', 0.0))
        sums[2] += float(infos[i].get('scaled_float_put', 0.0))
        sums[3] += int(infos[i].get('requested_calls_rounded_clipped', 0))
        sums[3] += int(infos[i].get('requested_puts_rounded_clipped', 0))
        sums[3] += int(infos[i].get('actual_calls_traded', 0))
        sums[3] += int(infos[i].get('actual_puts_traded', 0))
        sums[0] += float(infos[i].get('raw_pnl_deviation_abs', 0.0))
        sums[1] += float(infos[i].get('transaction_costs_total', 0.0))


def sb3_loop(dev, VecEnv, MON, envs=SB3_API_ENVS):
    """what the unchanged agents' host loop pays per step, infos included.
    sb3_loop: step_async + step_wait, then sb3_collect_pass (every row's get("episode") /
    get("is_success"), the done loop) -- Monitor on, the 3 Monitor keys; eval_loop: the same step
    with the 9 evaluation keys and eval_pass.  Each over whole steps; `pass_floor_us` is the same
    pass over plain dicts made beforehand from one step's rows (what those Python loops cost even
    if `infos` were a free list of dicts: the part no env can remove)."""
    out = dict(what="wall time per step of step_async + step_wait + the caller's per-step reads of infos "
                    "(SB3 collect_rollouts / the reference eval loop); Monitor on", sb3_loop={}, eval_loop={})
    rng = np.random.default_rng(5)
    for leg, keys in (("sb3_loop", MON), ("eval_loop", EVAL_INFO_KEYS)):
        for n in envs:
            # >= one episode end in the window at every n (episodes are 252 steps) for the SB3
            # pass; the eval pass at 65,536 reads 590k keys per step: fewer steps there
            steps = 260 if (leg == "sb3_loop" or n < 65536) else 24
            acts = rng.uniform(-1, 1, size=(4, n, 2)).astype(np.float32)
            env = VecEnv(n, mode="gbm", generate=GEN, seed=11, device=dev, monitor_keywords=MON, info_keys=keys,
                         **TRAIN_KW)
            env.reset()
            buf, sums = [], [0.0, 0.0, 0.0, 0]
            t_step, t_pass = np.empty(steps), np.empty(steps)
            for i in range(steps + 8):
                a = time.perf_counter()
                env.step_async(acts[i & 3])
                obs, rew, done, infos = env.step_wait()
                b = time.perf_counter()
                if leg == "sb3_loop":
                    sb3_collect_pass(infos, done, buf)
                else:
                    eval_pass(infos, n, sums)
                c = time.perf_counter()
                if i >= 8:
                    t_step[i - 8], t_pass[i - 8] = b - a, c - b
            plain = [dict(r) for r in infos]
            fl = []
            for _ in range(3):
                a = time.perf_counter()
                if leg == "sb3_loop":
                    sb3_collect_pass(plain, done, [])
                else:
                    eval_pass(plain, n, [0.0, 0.0, 0.0, 0])
                fl.append(time.perf_counter() - a)
            env.close()
            tot = t_step + t_pass
            out[leg][str(n)] = dict(
                us_per_step=round(float(tot.mean()) * 1e6, 2), us_median=round(float(np.median(tot)) * 1e6, 2),
                us_step_wait=round(float(t_step.mean()) * 1e6, 2), us_info_pass=round(float(t_pass.mean()) * 1e6, 2),
                pass_floor_us=round(float(np.median(fl)) * 1e6, 2), steps=steps,
                episodes_seen=len(buf) if leg == "sb3_loop" else None, keys=len(keys))
    return out


def _host_loop_timing(fn, steps, warm):
    for _ in range(warm):
        fn()
    ts = np.empty(steps)
    t0 = time.perf_counter()
    for i in range(steps):
        a = time.perf_counter()
        fn()
        ts[i] = time.perf_counter() - a
    wall = time.perf_counter() - t0
    return wall, ts


def policy_api(args, dev, K, stored_us, launches=100, warm_s=0.3):
    """Closed loop: he_rollout_policy, the reference's baseline policy evaluated on the env's own obs
    inside the rollout (baselines.py:77-103's policy_delta_every_step; on the LDS kernels with the
    policy in both lean / replay steppers), K steps per launch with obs / reward / done out, against
    the stored-action rollout of the same launch shape (`stored_us`)."""
    env = make_env(args, dev)
    n = env.num_envs
    obs = torch.empty((K, n, 13), dtype=torch.float32, device=dev)
    rew = torch.empty((K, n), dtype=torch.float32, device=dev)
    term = torch.empty((K, n), dtype=torch.uint8, device=dev)
    # warm until the clocks are back up after the env's construction (as the timed region's
    # MIN_WARMUP_SECONDS): batches of 20 launches for warm_s seconds
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(20):
            env.rollout_policy(K, "delta_every_step", None, obs, rew, term)
        torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(launches):
        env.rollout_policy(K, "delta_every_step", None, obs, rew, term)
    b.record()
    torch.cuda.synchronize(dev)
    us = a.elapsed_time(b) * 1e3 / launches
    env.close()
    # SURVEY 8(d)'s fused-rollout bytes without the 8-B action read (the policy makes it in the kernel)
    pol_bytes = n * (K * (SURVEY_ROLLOUT_B - 8) + SURVEY_ROLLOUT_STATE_B)
    gbs = pol_bytes / (us * 1e-6) / 1e9
    return dict(policy="delta_every_step", launches=launches, rollout_k=K, kernel_us=round(us, 3),
                value=round(n * K / us * 1e6, 1), unit="env-steps/s",
                vs_stored_actions=round(stored_us / us, 4) if stored_us else None,
                bytes_per_launch=int(pol_bytes), achieved_gbs=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4),
                what="device time per he_rollout_policy launch (HIP events around %d launches on the env's "
                     "stream): the actions come from the policy on each step's obs, not from memory" % launches)


def sb3_api(dev, classes=None, envs=SB3_API_ENVS, steps=504):
    """Wall time of the host paths the unchanged agents call:

    * `HedgingVecEnv.step_async` + `step_wait` with NumPy actions and NumPy results -- SB3's
      collect_rollouts (train_ppo_v2.py:127-141,204,230) -- at N = 2, 256 and 65,536, over
      `steps` steps (two whole episodes, so the episode-end work is averaged in), Monitor on;
      the same behind `DeviceVecNormalize` (train_ppo_v2.py:204) at N = 2 and 65,536;
    * the single `HedgingEnv.step` in a baselines.py:45-51-shaped loop (reset, policy, step,
      info.get(...) sums) over two episodes of policy_delta_every_step.

    `classes` = (HedgingVecEnv, HedgingEnv, DeviceVecNormalize, MONITOR_KEYWORDS) of the package
    to time (tools/sb3_time.py passes an older tree's for an A/B); default this tree's."""
    if classes is None:
        from cantorrl_amd.vec_env import HedgingVecEnv, MONITOR_KEYWORDS
        from cantorrl_amd.env import HedgingEnv
        from cantorrl_amd.vec_normalize import DeviceVecNormalize
        classes = (HedgingVecEnv, HedgingEnv, DeviceVecNormalize, MONITOR_KEYWORDS)
    VecEnv, Env, VecNorm, MON = classes
    out = dict(what="wall time per call of the host APIs the reference's agents drive (NumPy in, NumPy out): "
                    "step_async + step_wait per vector step, HedgingEnv.step per single-env step",
               vec_env={}, vecnorm={})
    rng = np.random.default_rng(7)
    for n in envs:
        acts = rng.uniform(-1, 1, size=(4, n, 2)).astype(np.float32)
        for wrap in (False, True):
            if wrap and n not in (envs[0], envs[-1]):
                continue
            env = VecEnv(n, mode="gbm", generate=GEN, seed=11, device=dev, monitor_keywords=MON, **TRAIN_KW)
            e = VecNorm(env, gamma=0.99) if wrap else env
            e.reset()
            k = [0]

            def one():
                e.step_async(acts[k[0] & 3])
                k[0] += 1
                return e.step_wait()

            wall, ts = _host_loop_timing(one, steps, 16)
            e.close()
            (out["vecnorm"] if wrap else out["vec_env"])[str(n)] = dict(
                us_per_step=round(wall / steps * 1e6, 2), us_median=round(float(np.median(ts)) * 1e6, 2),
                us_p99=round(float(np.percentile(ts, 99)) * 1e6, 2), env_steps_per_s=round(n * steps / wall, 1),
                steps=steps)
    env = Env(mode="gbm", generate=GEN, **TRAIN_KW)
    pnl = [0.0]

    def policy_delta_every_step(obs):
        # baselines.py:77-103: trade the option whose delta is usable towards zero book delta
        # (the caller's own per-step Python, the same work on either side of the swap)
        cd, pd = obs[7], obs[9]
        m = env.option_contract_multiplier
        tot = env.shares_held_fixed + (obs[3] * env.max_contracts_held * cd + obs[4] * env.max_contracts_held * pd) * m
        tc = tp = 0.0
        if abs(cd * m) > 1e-1:
            tc = -tot / (cd * m)
        elif abs(pd * m) > 1e-1:
            tp = -tot / (pd * m)
        lim = env.max_trade_per_step
        return np.array([np.clip(tc, -lim, lim), np.clip(tp, -lim, lim)], dtype=env.action_space.dtype)

    n_ep, t_steps = 2, 0
    t0 = time.perf_counter()
    for ep in range(n_ep + 1):
        if ep == 1:   # the first episode warms up
            t0, t_steps = time.perf_counter(), 0
        obs, _ = env.reset()
        term = trunc = False
        while not (term or trunc):
            obs, r, term, trunc, info = env.step(policy_delta_every_step(obs))
            pnl[0] += info.get("raw_pnl_deviation_abs", 0.0) + info.get("transaction_costs_total", 0.0)
            t_steps += 1
    wall = time.perf_counter() - t0
    env.close()
    out.update(sb3_loop(dev, VecEnv, MON, envs))
    out["single_env"] = dict(loop="baselines.py:32-56 evaluate_baseline_policy shape: reset, policy_delta_every_step, "
                                  "step, info.get sums", episodes=n_ep, steps=t_steps,
                             us_per_step=round(wall / t_steps * 1e6, 2), steps_per_s=round(t_steps / wall, 1),
                             reference_cpu_steps_per_s=REFERENCE_SINGLE_ENV_STEPS_S,
                             reference_note="the reference's hedging_env_v2.HedgingEnv.step on one core of the build "
                                            "container (SURVEY.md section 6), not timed on the GPU box")
    return out


# ---------------------------------------------------------------------- rbergomi workload
RB_MC, RB_DAYS = 5000, 252


def _rb_cpu_sample(seconds, base, seed=0, barrier=None):
    """One host core: the oracle's restatement of price_rbergomi_option_gpu
    (rbergomi_sim.py:261-306, NumPy FFTs) on batches of 8 options x 5000 MC paths."""
    from oracle import rbergomi_oracle as orc
    rng = np.random.default_rng(seed)
    B = 8
    S0 = np.full(B, base[0])
    K = np.round(S0)
    xi, H, eta, rho = (np.full(B, base[k]) for k in (1, 2, 3, 4))
    if barrier is not None:
        barrier.wait()
    n = 0
    t0 = time.perf_counter()
    while True:
        Z = rng.normal(size=(B, RB_MC, 32)) + 1j * rng.normal(size=(B, RB_MC, 32))
        orc.price_options(S0, K, 30 / 252, 0.04, xi, H, eta, rho, "call", Z, 1 / 252)
        n += B
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return n, el


def _rb_pool_task(a):
    return _rb_cpu_sample(a[0], a[1], a[2], _BARRIER)


def rb_cpu_baseline(seconds, base):
    """1 thread and one process per granted host core (forked before GPU init)."""
    import multiprocessing as mp
    n1, el1 = _rb_cpu_sample(seconds, base)
    procs, avail, why = host_cores()
    ctx = mp.get_context("fork")
    b = ctx.Barrier(procs)
    with ctx.Pool(procs, initializer=_pool_init, initargs=(b,)) as pool:
        res = pool.map(_rb_pool_task, [(seconds, tuple(base), i + 1) for i in range(procs)])
    return dict(value=sum(n / e for n, e in res), unit="options/s", cores=procs, affinity_cores=avail,
                cores_source=why, kind="port",
                sample=f"oracle/rbergomi_oracle.py price_options (the reference's FFT form), batches of 8 options x "
                       f"{RB_MC} MC paths, {procs} processes x {seconds:.0f} s (NumPy, 1 thread each)",
                single_core_value=n1 / el1,
                single_core_sample=f"{n1} options in {el1:.1f} s, 1 thread")


def rb_roofline(valu, traffic, kern_ms, n_opt):
    """mc_kernel's roofline: VALU issue.  `achieved` = VALU wave-instructions per SIMD-cycle
    (SQ_INSTS_VALU over GRBM_GUI_ACTIVE / 8 cycles x 1,024 SIMDs), `peak` = the issue bound of
    the kernel's own f64 / other mix (a wave64 instruction every 2 cycles per SIMD, f64 every 4),
    plus its f64 FLOP rate against the 78.6 TF vector peak; `traffic` = HBM bytes per launch
    from the PMC pass (about 7 f64 per option -- the path's parameters, S and v in, the mark
    out: negligible against the 5,000 x 30 Euler steps behind each mark)."""
    v, note = valu
    out = dict(bound="valu", unit="VALU wave-instructions per SIMD-cycle", achieved=None, peak=None, frac=None,
               traffic=None, kernel="mc_kernel (rb_price_atm_marks)", kernel_us=round(kern_ms * 1e3, 1),
               algorithmic_bytes_per_launch=int(n_opt * 7 * 8))
    if v is not None:
        out.update(achieved=v["issue_per_simd_cycle"], peak=v["issue_bound_per_simd_cycle"], frac=v["valu_issue_frac"],
                   f64_share=v["f64_share"], valu_insts=v["valu_insts"])
        tf = v["f64_flop"] / (kern_ms * 1e-3) / 1e12
        out.update(f64_tflops=round(tf, 3), f64_frac_of_vector_peak=round(tf / FP64_VECTOR_PEAK_TFLOPS, 4),
                   peak_f64_tflops=FP64_VECTOR_PEAK_TFLOPS)
    else:
        out["valu_note"] = note
    if traffic[0] is not None:
        out["traffic"] = int(traffic[0])
        out["traffic_counters"] = {k: round(x, 1) for k, x in traffic[1].items()}
    else:
        out["traffic_note"] = traffic[1]
    return out


def rbergomi_main(args):
    """One step = one rb_price_atm_marks launch: rolling-ATM call and put marks for
    every (path, day) of args.rb_paths paths x 252 days, 5000 MC paths x 30 Euler
    steps each (rbergomi_sim.py:404-451, all days at once)."""
    from cantorrl_amd import rbergomi as rb
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    hist = np.load(os.path.join(REPO, "tests", "golden", "rb_estimate.npz"))["hist__prices"]
    base = rb.estimate_base_params(hist)
    cpu = None
    valu, traffic = (None, "skipped"), (None, "skipped")
    if world == 1 and not args.probe and not args.no_pmc:
        # counters of mc_kernel in rocprofv3 children (before this process touches the GPU)
        pa = ["--workload", "rbergomi", "--rb-paths", str(args.rb_paths), "--rb-normals", args.rb_normals]
        res, err = pmc_pass(args, VALU_COUNTERS, "mc_kernel", probe_argv=pa)
        valu = (valu_summary(res).get("mc_kernel"), None) if res else (None, err)
        traffic = pmc_traffic(args, "mc_kernel", pa)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.probe:
        cpu = rb_cpu_baseline(args.cpu_seconds, base)
    dist = None
    if world > 1:
        dist, _ = init_dist(local)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    P = args.rb_paths
    cfg = rb.make_config(P, path_offset=rank * P, normals=args.rb_normals)
    params = rb.sample_params(cfg, base, dev)
    paths, vol = rb.simulate_paths(cfg, params, dev)
    call = torch.empty((P, RB_DAYS), dtype=torch.float64, device=dev)
    put = torch.empty_like(call)
    lib = rb.load()
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    ptrs = [ctypes.c_void_p(t.data_ptr()) for t in (params, paths, vol, call, put)]

    def launch():
        st = lib.rb_price_atm_marks(ctypes.byref(cfg), *ptrs, sp)
        if st != 0:
            raise RuntimeError(lib.rb_last_error().decode())

    if args.probe:   # the PMC passes' program: two launches
        for _ in range(2):
            launch()
        torch.cuda.synchronize()
        return
    # one launch prices 1M options (~1 s in f64): a handful of launches, not the env's 25,600
    K = max(1, 5 if args.steps is None else args.steps)
    W = max(0, 1 if args.warmup is None else args.warmup)
    for _ in range(W):
        launch()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    hev = HipEvents()
    e0, e1 = hev.create(), hev.create()
    t0 = time.perf_counter()
    hev.record(e0, stream)
    for _ in range(K):
        launch()
    hev.record(e1, stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = hev.elapsed_ms(e0, e1) / K
    hev.destroy(e0, e1)
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    n_opt = P * RB_DAYS * 2
    if rank == 0:
        line = {
            "metric": "rolling-ATM MC option marks/sec (rBergomi generator, rbergomi_sim.py)",
            "value": round(n_opt * world * K / wall, 1),
            "unit": "options/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(wall * 1e3 / K, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.rb_normals == "f64" else "f64 (f32-precision normals)",
            "data": "synthetic (rBergomi parameters estimated from data/historical_prices.csv, perturbed per path; "
                    "Philox4x32-10 normals)",
            "config": {"workload": f"generate_paths_and_options marks: {P} paths/GPU x {RB_DAYS} days x "
                                   f"{{call, put}}, {RB_MC} MC paths x 30 Euler steps each",
                       "paths_per_gpu": P, "n_mc": RB_MC, "normals": args.rb_normals,
                       "parallelism": f"path-shard x{world}"},
            "kernel": {"name": "mc_kernel (rb_price_atm_marks)", "ms_per_launch": round(kern_ms, 3),
                       "options_per_s": round(n_opt / (kern_ms * 1e-3), 1),
                       "mc_path_steps_per_s": round(n_opt * RB_MC * 30 / (kern_ms * 1e-3), 1),
                       "bound": "valu (f64 FMA / exp, Philox): no HBM traffic to speak of "
                                "(5 f64 in, 1 f64 out per option)"},
            "full_dataset_s": round(100000 * RB_DAYS * 2 / (n_opt * world * K / wall), 2),
            "roofline": rb_roofline(valu, traffic, kern_ms, n_opt),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    rank_phase("done")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launcher_cmd(argv, n, port):
    """The child command of `bench.py --gpus N` (N > 1): one rank per GPU on this node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch(args, argv):
    """`--gpus N` without WORLD_SIZE: this process makes no GPU call.  It runs the PMC pass
    (a rocprofv3 child on one GPU) and the CPU baseline, starts the N ranks as a child
    process (never exec), hands its results to rank 0 through a file, and returns the
    child's exit status."""
    import subprocess
    import tempfile
    parent = dict(pmc=None, pmc_note="skipped", cpu_baseline=None)
    if not args.launch_dry_run:
        if args.workload == "env" and not args.no_pmc:
            t, v = pmc_traffic(args)
            parent.update(pmc=t, pmc_note=v if t is None else None, pmc_counters=v if t is not None else None)
            vv, note = pmc_valu(args)
            parent.update(valu=vv, valu_note=note)
        if not args.no_cpu_baseline:
            parent["cpu_baseline"] = (cpu_baseline(args.cpu_seconds) if args.workload == "env"
                                      else None)
    fd, path = tempfile.mkstemp(prefix="bench_parent_", suffix=".json", dir="/tmp")
    with os.fdopen(fd, "w") as fh:
        json.dump(parent, fh)
    status_dir = tempfile.mkdtemp(prefix="bench_ranks_", dir="/tmp")
    cmd = launcher_cmd(argv, args.gpus, free_port())
    env = dict(os.environ, BENCH_PARENT_RESULTS=path, BENCH_RANK_STATUS_DIR=status_dir)
    try:
        if args.launch_dry_run:
            print(json.dumps(dict(cmd=cmd, parent_results=path, cuda_initialized=torch.cuda.is_initialized())),
                  flush=True)
            return 0
        # the child in a session of its own, so a wall-limit kill takes its whole process group
        # (torch.distributed.run and every rank) and nothing else
        proc = subprocess.Popen(cmd, env=env, start_new_session=True)
        try:
            rc = proc.wait(timeout=LAUNCH_TIMEOUT_S)
            why = None if rc == 0 else f"exit status {rc}"
        except subprocess.TimeoutExpired:
            import signal
            for sig, grace in ((signal.SIGTERM, 15), (signal.SIGKILL, 15)):
                try:
                    os.killpg(proc.pid, sig)
                except ProcessLookupError:
                    break
                try:
                    proc.wait(timeout=grace)
                    break
                except subprocess.TimeoutExpired:
                    continue
            rc, why = 124, f"wall limit {LAUNCH_TIMEOUT_S:g} s (BENCH_LAUNCH_TIMEOUT)"
        if why is not None:
            report_ranks(status_dir, args.gpus, why)
        return rc
    finally:
        os.unlink(path)
        import shutil
        shutil.rmtree(status_dir, ignore_errors=True)


def report_ranks(status_dir, world, why):
    """After a failed or timed-out `--gpus N` child: each rank's last recorded phase, and the
    ranks that never reached "done" named, on stderr and as one JSON line on stdout."""
    last = {}
    for r in range(world):
        f = os.path.join(status_dir, f"rank{r}")
        lines = open(f).read().splitlines() if os.path.exists(f) else []
        last[r] = lines[-1].split(" ", 1)[1] if lines else "no record (never started)"
    stalled = [r for r in range(world) if last[r] != "done"]
    for r in range(world):
        print(f"[bench launcher] rank {r}: last phase: {last[r]}", file=sys.stderr, flush=True)
    print(f"[bench launcher] FAILED ({why}); ranks not done: {stalled}", file=sys.stderr, flush=True)
    print(json.dumps(dict(error="bench --gpus %d failed: %s" % (world, why), ranks_not_done=stalled,
                          last_phase={str(r): last[r] for r in range(world)})), flush=True)


def parent_results():
    """What the `--gpus N` launcher measured (rank 0 merges it), or None."""
    p = os.environ.get("BENCH_PARENT_RESULTS")
    if not p or not os.path.exists(p):
        return None
    with open(p) as fh:
        return json.load(fh)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.envs is None and args.workload == "env":
            args.envs = CONFIGS[args.config]["envs"]
        if args.rollout_k is None and args.workload == "env":
            lds0 = args.mode == "rollout" and lds_rollout(CONFIGS[args.config])
            args.rollout_k = 256 if (lds0 or CONFIGS[args.config]["mode"] == "replay") else M_BLOCK
        sys.exit(launch(args, argv))
    if args.dist_selftest:
        dist_selftest()
        return
    if args.workload == "rbergomi":
        rbergomi_main(args)
        return
    if args.envs is None:
        args.envs = CONFIGS[args.config]["envs"]
    lds = args.mode == "rollout" and lds_rollout(CONFIGS[args.config])
    replay = CONFIGS[args.config]["mode"] == "replay"  # one step_kernel dispatch per he_rollout, any K
    if args.rollout_k is None:
        args.rollout_k = 256 if (lds or replay) else M_BLOCK
    if args.mode == "rollout" and (args.rollout_k < 1 or (not (lds or replay) and args.rollout_k > M_BLOCK)):
        raise SystemExit("--rollout-k must be >= 1 (<= 64 on the tile path: one dispatch per call is timed)")
    if args.probe:
        probe(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pmc = (None, "skipped")
    valu = (None, "skipped")
    step_pmc = (None, "skipped")
    cpu = None
    has_book = bool(CONFIGS[args.config]["gen"].get("book"))
    parent = parent_results()
    if parent is not None:  # ranks of a `--gpus N` launch: the launcher measured these
        pmc = (parent["pmc"], parent.get("pmc_counters") or parent.get("pmc_note"))
        valu = (parent.get("valu"), parent.get("valu_note"))
        cpu = parent["cpu_baseline"]
    elif world == 1:
        if not args.no_pmc:
            pmc = pmc_traffic(args)
            # the instruction-issue side: the LDS kernel makes the market on chip, so every
            # configuration is partly VALU-bound (with a book or Heston, mostly)
            valu = pmc_valu(args)
            if args.mode != "graph" and not args.no_step_api:
                # the step_api line's kernel (he_step -> step1_kernel): its own HBM traffic
                import copy
                ga = copy.copy(args)
                ga.mode = "graph"
                step_pmc = pmc_traffic(ga)
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds)   # before the GPU is touched (forks workers)
    dist, backend = None, None
    if world > 1:
        dist, backend = init_dist(local)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = CONFIGS[args.config]
    n = args.envs

    acts = bench_actions(n, rank, dev, args.action_sets)
    stream = torch.cuda.Stream(device=dev)
    gathered = (torch.empty((world * n, 4), dtype=torch.float32, device=dev if backend == "nccl" else "cpu")
                if world > 1 else None)

    env = make_env(args, dev, rank)
    runner = Runner(args, env, args.mode, acts, stream, dist, gathered)
    acts = runner.acts   # [256, n, 2]: set 0 (the other legs below use one set)
    # at least two full episodes (504 steps) in the timed window
    K = -(-max(args.steps, MIN_TIMED_STEPS) // runner.chunk) * runner.chunk
    W = -(-args.warmup // runner.chunk) * runner.chunk
    rank_phase("env made; warmup %d + timed %d steps" % (W, K))
    wall, dev_ms = timed(runner, K, W, dist)
    rank_phase("timed region done")
    shard = None
    if args.mode == "rollout":
        # every env's summaries after the last launch, gathered in global env order (outside
        # the timed region), then each rank's re-run of its neighbour's last envs
        with torch.cuda.stream(stream):
            final = env.episode_summaries()
            if dist is not None:
                allg = torch.empty((world * n, 4), dtype=torch.float32, device=gathered.device)
                gather_summaries(dist, final, allg)
            else:
                allg = final
        torch.cuda.synchronize()
        nb, j0, m = shard_check_slice(rank, world, n)
        got = shard_check_run(args, dev, stream, runner.runs, nb, j0, m)
        shard = shard_check_verdict(dist, got, allg, nb, j0, n, device="cpu" if backend == "gloo" else dev)
        rank_phase("shard check: %s" % shard.get("result") if isinstance(shard, dict) else "shard check")
    payload = None
    if dist is not None:
        payload = dict(what="he_episode_summaries: per-env {return, sum P&L, sum cost, length} f32 [envs, 4], "
                            "all-gathered to [world * envs, 4]", backend="rccl" if backend == "nccl" else backend,
                       every_steps=GATHER_EVERY,
                       bytes_per_rank=n * 16, gathers=runner.gathers)
        if backend != "nccl":
            payload["sync"] = ("host-synced rehearsal: gather_summaries copies the device summaries to the host "
                               "(local.to(cpu), a stream sync) and gathers them over gloo; the boundary time "
                               "measures that host round trip, not RCCL")
        payload.update(summarize_payload(runner.gathered))
        if args.gather_rollout and runner.rollout_gathered is not None:
            ro, rr, rt = runner.rollout_gathered
            payload["rollout_tensors"] = dict(
                what="the last he_rollout's obs / reward / terminated [K, N, ...] of every rank, gathered along the "
                     "env dimension into [K, world * N, ...] (global env order, cantorrl_amd.dist.gather_rollout "
                     "env_dim=1)", shapes=[list(ro.shape), list(rr.shape), list(rt.shape)],
                bytes_per_rank=int(sum(t.numel() * t.element_size() for t in (ro, rr, rt)) // world))
    hev = HipEvents()
    probe_ms = kernel_time_ms(hev, runner, 64 if args.mode == "rollout" else 256)
    env.close()
    # The dominant kernel's average launch duration.  On the LDS path one he_rollout is one
    # lds_rollout_kernel dispatch, so the HIP events around the timed region on the
    # launching stream, over its launches, are that average (the task's definition; at one
    # rank nothing else runs on the stream).  Elsewhere (tile path: market + step kernels
    # per call; ranks > 1: the gathers ride on the stream) the per-dispatch probe
    # (he_time_next_step: hipExtLaunchKernelGGL events around exactly the step kernel).
    launches = K // runner.chunk
    region = (lds or (replay and args.mode == "rollout")) and world == 1
    kern_ms = dev_ms / launches if region else probe_ms
    per_rank = None
    if dist is not None:
        # every rank's own timers, so an N-rank line explains itself: the step kernel's
        # per-dispatch probe, the device time per launch over the timed region (kernels +
        # the boundaries riding on the stream), and the boundary's device time
        b_us, r_us = runner.boundary_us()
        mine = torch.tensor([rank, probe_ms * 1e3, dev_ms / launches * 1e3,
                             b_us if b_us is not None else float("nan"), r_us if r_us is not None else float("nan"),
                             runner.gathers, wall], dtype=torch.float64,
                            device="cpu" if backend == "gloo" else dev)
        allv = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        per_rank = []
        for v in allv:
            v = v.cpu().tolist()
            per_rank.append(dict(rank=int(v[0]), kernel_us_probe=round(v[1], 3), device_us_per_launch=round(v[2], 3),
                                 boundary_us=None if v[3] != v[3] else round(v[3], 2),
                                 rollout_gather_us=None if v[4] != v[4] else round(v[4], 2),
                                 boundaries=int(v[5]), wall_s=round(v[6], 6)))

    roof = roofline(args.mode, n, kern_ms, args.rollout_k, has_book, tile_layout(cfg["mode"], n), lds)
    roof["kernel_us_source"] = ("HIP events around the timed region / %d launches" % launches if region else
                                "he_time_next_step probe: HIP events around single dispatches")
    roof["kernel_us_probe"] = round(probe_ms * 1e3, 3)
    roof["kernel_us_timed_region"] = round(dev_ms / launches * 1e3, 3)
    if not lds and not replay:  # the tile path: market_kernel makes the HBM market tile
        roof["tile_layout"] = tile_layout(cfg["mode"], n)
        mkt_ms = market_time_ms(hev, args, dev, acts, stream)
        roof["market_kernel_us_per_64_steps"] = round(mkt_ms * 1e3, 3)
        roof["market_kernel_us_per_step"] = round(mkt_ms * 1e3 / M_BLOCK, 3)
        steps_per_launch = args.rollout_k if args.mode == "rollout" else 1
        if mkt_ms / M_BLOCK > kern_ms / steps_per_launch:
            roof["dominant_kernel"] = "market_kernel (the HBM market tile, %.1f us per step vs %.1f for the steps)" % (
                mkt_ms * 1e3 / M_BLOCK, kern_ms * 1e3 / steps_per_launch)
    roof = finish_roofline(roof, cfg, valu, pmc, kern_ms)

    step_api = None
    if world == 1 and args.mode != "graph" and not args.no_step_api:
        # secondary: the Gym step API path, one he_step launch per step in hipGraphs
        env_g = make_env(args, dev)
        rg = Runner(args, env_g, "graph", acts, stream)
        Kg = -(-min(K, 2560) // M_BLOCK) * M_BLOCK
        wall_g, _ = timed(rg, Kg, M_BLOCK * 4, None)
        kg = kernel_time_ms(hev, rg, 256)
        env_g.close()
        rf = roofline("graph", n, kg, 1, has_book, tile_layout(cfg["mode"], n))
        step_api = step_api_line(n, Kg, wall_g, rf, step_pmc, tile_layout(cfg["mode"], n))

    sb3 = None
    if world == 1 and args.config == 2 and not args.no_sb3_api:
        sb3 = sb3_api(dev)
    pol = None
    if world == 1 and args.mode == "rollout" and not args.no_policy_api:
        pol = policy_api(args, dev, args.rollout_k, kern_ms * 1e3)

    if rank == 0:
        line = {
            "metric": "env-steps/sec (batched episodes)",
            "value": round(n * world * K / wall, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": runner.warmup_steps,
            # the command's --steps / --warmup: raised to the timed floor (MIN_TIMED_STEPS, >= 2
            # episodes and 100 launches) and to whole launches of the rollout chunk
            "requested_steps": args.steps,
            "requested_warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / K, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+f32",
            "data": ("synthetic (a 100,000 x 253 GBM / lognormal-variance table with rolling-ATM BS marks in "
                     "the reference NPZ layout, U(-1,1) actions pre-generated on device)" if replay else
                     "synthetic (GBM paths from Philox4x32-10, U(-1,1) actions pre-generated on device)"),
            "config": {"workload": cfg["workload"], "config_index": args.config, "envs_per_gpu": n,
                       "episode_length": (cfg["table"]["cols"] - 1) if replay else cfg["gen"]["episode_length"],
                       "mode": args.mode,
                       "rollout_k": args.rollout_k if args.mode == "rollout" else None,
                       "action_sets": args.action_sets,
                       "parallelism": f"env-shard x{world}"},
            "device_ms_per_step": round(dev_ms / K, 6),
            "roofline": roof,
            "step_api": step_api,
            "sb3_api": sb3,
            "policy_api": pol,
            "shard_check": shard,
            "cpu_baseline": cpu,
        }
        if payload is not None:
            line["gather"] = payload
            line["per_rank"] = per_rank
            bu = [r["boundary_us"] for r in per_rank if r["boundary_us"] is not None]
            if bu:
                payload["boundary_us_per_256_steps"] = dict(
                    max=max(bu), mean=round(sum(bu) / len(bu), 2),
                    what="device time on the launching stream of he_episode_summaries + the all-gather, per "
                         "rollout-buffer boundary (every %d steps), the timed region's boundaries" % GATHER_EVERY)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    rank_phase("done")


if __name__ == "__main__":
    main()
