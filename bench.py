#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the batched hedging env on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--mode graph|eager|rollout]

Workload = BASELINE.json configs[1]: 65,536 parallel envs per GPU, GBM price
advance (Philox4x32-10 normals), Black-Scholes rolling-ATM marks, v2 env with
the train_ppo_v2.py reward settings (abs loss, w=1e-3, lambda=1e-4,
theta=2e-4, 1 bp slippage).  One "step" = one env-step of every env: actions
[N,2] in (pre-generated, HBM-resident), obs [N,13] / reward [N] / done flags
out, auto-reset inside the kernel.

Modes: `graph` (default) replays he_step launches captured into a hipGraph,
one kernel per step; `eager` calls he_step from Python every step; `rollout`
fuses 64 steps per launch (he_rollout).  For N>1 the script runs under
torch.distributed.run, one rank per GPU (weak scaling: E envs per rank, env
ids offset by rank), and all-gathers per-env rewards over RCCL every 256 steps
(the rollout-buffer boundary of train_ppo_v2.py:48).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# algorithmic HBM bytes per env-step of step_kernel<GBM> (DESIGN.md "Roofline"):
#   reads : state (t 4, pos 4, cash 8) 16 + action 8 + market tile slots
#           (pre {S,v,C,P} 16, post {S,v,C,P} 16, post greeks 16) 48            = 72
#   writes: state 16 + obs 52 + reward 4 + terminated 1 + truncated 1             = 74
STEP_BYTES_PER_ENV = 146
# market_kernel per env-step: tile {S,v,C,P} + greeks written (32) + per-block state
MARKET_BYTES_PER_ENV = 32
# he_rollout per env-step: action 8 + obs 52 + reward 4 + terminated 1 + tile read 32
ROLLOUT_BYTES_PER_ENV = 97
ROLLOUT_STATE_BYTES = 16 + 16 + 16
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

TRAIN_KW = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002,
                slippage_bps=1.0)  # train_ppo_v2.py:74-80
GEN = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=252)

# BASELINE.json configs (configs[0] is the CPU case = cpu_baseline below)
CONFIGS = {
    2: dict(envs=65536, mode="gbm", gen=GEN, kw=TRAIN_KW,
            workload="configs[1]: 65,536 parallel envs/GPU, European call (BS rolling-ATM marks), GBM, "
                     "v2 env, train_ppo_v2 reward"),
    3: dict(envs=1048576, mode="gbm", gen=GEN, kw=dict(TRAIN_KW, slippage_bps=5.0),
            workload="configs[2]: 1,048,576 parallel envs/GPU, European call, GBM, proportional costs "
                     "(5 bp slippage + $0.65 commission)"),
    5: dict(envs=131072, mode="heston",
            gen=dict(GEN, heston_kappa=2.0, heston_theta=0.029028, heston_xi=0.3, heston_rho=-0.7),
            kw=TRAIN_KW,
            workload="configs[4] market: Heston full-truncation Euler (rho=-0.7), 131,072 envs/GPU "
                     "(1M over 8 GPUs)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2520)
    ap.add_argument("--warmup", type=int, default=256)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS), help="BASELINE.json config")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the config's)")
    ap.add_argument("--mode", choices=["graph", "eager", "rollout"], default="graph")
    ap.add_argument("--graph-chunk", type=int, default=64)
    ap.add_argument("--rollout-k", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic pass")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def cpu_baseline(seconds):
    """The oracle (NumPy restatement of the reference env) on host cores, N=256."""
    from oracle.hedging_oracle import OracleVecEnv
    n = 256
    env = OracleVecEnv(n, mode="gbm", gen=dict(GEN, seed=42), **TRAIN_KW)
    env.seed_envs_at(np.arange(n), [42] * n)
    env.reset()
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, size=(64, n, 2)).astype(np.float32)
    for k in range(8):
        env.step(acts[k])
    steps = 0
    t0 = time.perf_counter()
    while True:
        env.step(acts[steps % 64])
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return dict(value=n * steps / el, unit="env-steps/s", cores=1, kind="port",
                sample=f"oracle/hedging_oracle.py OracleVecEnv GBM, 256 envs x {steps} steps "
                       f"({el:.1f} s, 1 thread, NumPy)")


def probe(args):
    """Short run for counter collection: 2 market blocks of eager he_step."""
    torch.cuda.set_device(0)
    from cantorrl_amd.vec_env import HedgingVecEnv
    cfg = CONFIGS[args.config]
    n = args.envs
    env = HedgingVecEnv(n, mode=cfg["mode"], generate=cfg["gen"], seed=args.seed, return_numpy=False,
                        info_keys=(), **cfg["kw"])
    env.reset_tensors()
    acts = torch.rand((64, n, 2), device="cuda:0") * 2 - 1
    for k in range(128):
        env.step_tensors(acts[k % 64])
    torch.cuda.synchronize()
    env.close()


def pmc_traffic(args):
    """HBM bytes per step_kernel launch from rocprofv3 PMC counters, one counter per
    pass (MI355X_MICROARCH.md "HBM": FETCH_SIZE reads 1/2 of a wide coalesced read on
    gfx950, so bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024).  Runs BEFORE this process
    touches the GPU; the profiled program is a child (`rocprofv3 ... -- python3`)."""
    import csv
    import re
    import glob
    import shutil
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir="/tmp") as td:
            cmd = ["rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", td, "-o", "pmc", "--",
                   sys.executable, os.path.abspath(__file__), "--probe", "--envs", str(args.envs),
                   "--config", str(args.config)]
            try:
                subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                               timeout=240, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
            except Exception as e:  # noqa: BLE001
                return None, f"rocprofv3 --pmc {ctr} failed: {e}"
            rows = []
            for f in glob.glob(os.path.join(td, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for r in csv.DictReader(fh):
                        if re.search(r"step1?_kernel", r.get("Kernel_Name", "")) and r.get("Counter_Name") == ctr:
                            rows.append(float(r["Counter_Value"]))
            if not rows:
                return None, f"no {ctr} rows for step_kernel"
            vals[ctr] = float(np.mean(rows[8:] if len(rows) > 16 else rows))
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, vals


def main():
    args = parse()
    if args.envs is None:
        args.envs = CONFIGS[args.config]["envs"]
    if args.probe:
        probe(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    pmc = (None, "skipped")
    if world == 1 and not args.no_pmc and args.mode != "rollout":
        pmc = pmc_traffic(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from cantorrl_amd.vec_env import HedgingVecEnv
    cfg = CONFIGS[args.config]
    n = args.envs
    env = HedgingVecEnv(n, mode=cfg["mode"], generate=cfg["gen"], seed=args.seed, global_env_offset=rank * n,
                        device=dev, return_numpy=False, info_keys=(), **cfg["kw"])
    env.reset_tensors()
    ring = 256
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    acts = torch.rand((ring, n, 2), device=dev, generator=g) * 2 - 1
    stream = torch.cuda.Stream(device=dev)
    gathered = torch.empty((world, n), dtype=torch.float32, device=dev) if world > 1 else None

    lib = env.lib
    h = env._h
    obs, rew, term, trunc, tobs = env._obs, env._rew, env._term, env._trunc, env._tobs

    def launch(k, s):
        st = lib.he_step(h, acts[k % ring].data_ptr(), obs.data_ptr(), rew.data_ptr(), term.data_ptr(),
                         trunc.data_ptr(), tobs.data_ptr(), None, s)
        if st:
            raise RuntimeError(lib.he_last_error(h).decode())

    K = args.steps
    W = args.warmup
    graphs = []
    if args.mode == "graph":
        C = args.graph_chunk  # == market block: every graph = one block of steps
        K = -(-K // C) * C
        W = -(-W // C) * C
        with torch.cuda.stream(stream):
            # one eager block first, so each captured graph is the steady state
            # [fork: market_kernel(b+1) on the side stream || C x step_kernel(b)] + join
            for j in range(C):
                launch(j, stream.cuda_stream)
            env.sync_market()
            torch.cuda.synchronize()
            for gi in range(ring // C):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=stream):
                    cs = torch.cuda.current_stream().cuda_stream
                    for j in range(C):
                        launch(gi * C + j, cs)
                    env.sync_market()
                graphs.append(gr)
        torch.cuda.synchronize()
        # device state = after the eager block; graphs replay in capture order from here

    roll_obs = roll_rew = roll_term = None
    if args.mode == "rollout":
        RK = args.rollout_k
        roll_obs = torch.empty((RK, n, 13), dtype=torch.float32, device=dev)
        roll_rew = torch.empty((RK, n), dtype=torch.float32, device=dev)
        roll_term = torch.empty((RK, n), dtype=torch.uint8, device=dev)

    replays = [0]

    def run(steps, s):
        """Enqueue `steps` env-steps on stream s."""
        done = 0
        cs = s.cuda_stream
        while done < steps:
            if args.mode == "graph":
                # K, W are multiples of the chunk; graphs replay in capture order
                graphs[replays[0] % len(graphs)].replay()
                replays[0] += 1
                done += args.graph_chunk
            elif args.mode == "eager":
                launch(done, cs)
                done += 1
            else:
                RK = min(args.rollout_k, steps - done)
                a0 = (done % ring)
                a = acts[a0:a0 + RK] if a0 + RK <= ring else acts[:RK]
                st = lib.he_rollout(h, RK, a.data_ptr(), roll_obs.data_ptr(), roll_rew.data_ptr(),
                                    roll_term.data_ptr(), cs)
                if st:
                    raise RuntimeError(lib.he_last_error(h).decode())
                done += RK
            if dist is not None and done % 256 == 0:
                dist.all_gather_into_tensor(gathered, rew)

    with torch.cuda.stream(stream):
        run(W, stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        run(K, stream)
        ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    dev_ms = ev0.elapsed_time(ev1)

    # live per-launch kernel duration: HIP events bracketing single launches on `stream`
    # (the he_step of every 64th step also launches market_kernel for the next 64 steps)
    # `kev` brackets exactly the step_kernel dispatch (he_time_next_step ->
    # hipExtLaunchKernelGGL), `oev` the whole call (+ market_kernel every 64 steps)
    nprobe = 256
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")  # the HIP runtime torch (and libhedgeenv) use

    def mk():
        e = ctypes.c_void_p()
        if hip.hipEventCreate(ctypes.byref(e)) != 0:
            raise RuntimeError("hipEventCreate failed")
        return e

    def elapsed(a, b):
        ms = ctypes.c_float()
        if hip.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    kev = [(mk(), mk()) for _ in range(nprobe)]
    oev = [(mk(), mk()) for _ in range(nprobe)]
    env.reset_tensors()
    torch.cuda.synchronize()
    sh = ctypes.c_void_p(stream.cuda_stream)
    with torch.cuda.stream(stream):
        for k in range(nprobe):
            hip.hipEventRecord(oev[k][0], sh)
            lib.he_time_next_step(h, kev[k][0], kev[k][1])
            if args.mode == "rollout":
                RK = args.rollout_k
                lib.he_rollout(h, RK, acts[:RK].data_ptr(), roll_obs.data_ptr(), roll_rew.data_ptr(),
                               roll_term.data_ptr(), stream.cuda_stream)
            else:
                launch(k, stream.cuda_stream)
            hip.hipEventRecord(oev[k][1], sh)
    torch.cuda.synchronize()
    kd = np.array([elapsed(a, b) for a, b in kev])  # ms
    od = np.array([elapsed(a, b) for a, b in oev])
    for a, b in kev + oev:
        hip.hipEventDestroy(a)
        hip.hipEventDestroy(b)
    M = 64
    if args.mode == "rollout":
        kern_ms = float(np.mean(kd[4:]))
        mkt_ms = None  # prefetched on the side stream (see graph-mode probe)
    else:
        idx = np.arange(8, nprobe)
        kern_ms = float(np.mean(kd[idx]))
        # market_kernel is prefetched on the library's side stream here; time it on a
        # handle without prefetch, where it runs inside the he_step of a block boundary
        env2 = HedgingVecEnv(n, mode=cfg["mode"], generate=cfg["gen"], seed=args.seed, device=dev,
                             return_numpy=False, info_keys=(), market_prefetch=False, **cfg["kw"])
        env2.reset_tensors()
        m = []
        with torch.cuda.stream(stream):
            for k in range(4 * M):
                a, b = mk(), mk()
                hip.hipEventRecord(a, sh)
                st2 = lib.he_step(env2._h, acts[k % ring].data_ptr(), env2._obs.data_ptr(), env2._rew.data_ptr(),
                                  env2._term.data_ptr(), env2._trunc.data_ptr(), None, None, stream.cuda_stream)
                hip.hipEventRecord(b, sh)
                if st2:
                    raise RuntimeError(lib.he_last_error(env2._h).decode())
                m.append((a, b))
        torch.cuda.synchronize()
        d2 = np.array([elapsed(a, b) for a, b in m])
        for a, b in m:
            hip.hipEventDestroy(a)
            hip.hipEventDestroy(b)
        mkt_ms = float(np.median(d2[M::M])) - float(np.median(np.delete(d2, np.arange(0, 4 * M, M))))
        env2.close()

    total_envs = n * world
    value = total_envs * K / wall
    if args.mode == "rollout":
        RK = args.rollout_k
        bytes_launch = n * RK * (ROLLOUT_BYTES_PER_ENV + ROLLOUT_STATE_BYTES / RK)
        kname = "step_kernel<GBM> (K=%d fused) + market_kernel" % RK
    else:
        bytes_launch = n * STEP_BYTES_PER_ENV
        kname = "step_kernel<GBM> (K=1)"
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None, kernel=kname,
                kernel_us=round(kern_ms * 1e3, 3), bytes_per_launch=int(bytes_launch))
    if mkt_ms is not None:
        roof["market_kernel_us_per_64_steps"] = round(mkt_ms * 1e3, 3)
        roof["market_kernel_us_per_step"] = round(mkt_ms * 1e3 / M, 3)
    if pmc[0] is not None:
        roof["traffic"] = int(pmc[0])
        roof["traffic_counters_kb"] = {k: round(v, 1) for k, v in pmc[1].items()}
    else:
        roof["traffic_note"] = pmc[1]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        line = {
            "metric": "env-steps/sec (batched episodes)",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(wall * 1e3 / K, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+f32",
            "data": "synthetic (GBM paths from Philox4x32-10, U(-1,1) actions pre-generated on device)",
            "config": {"workload": cfg["workload"], "config_index": args.config, "envs_per_gpu": n,
                       "episode_length": cfg["gen"]["episode_length"], "mode": args.mode,
                       "parallelism": f"env-shard x{world}"},
            "device_ms_per_step": round(dev_ms / K, 6),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    env.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
