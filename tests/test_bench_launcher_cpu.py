"""bench.py's N>1 path on CPU: the `--gpus N` launcher builds the
torch.distributed.run command for N ranks and never touches the GPU itself, and the
per-env episode-summary all-gather (bench.gather_summaries, the code the ranks run at
every 256-step boundary) over gloo at world size 2 equals one process holding every env.
"""
import importlib.util
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle.hedging_oracle import OracleVecEnv

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launcher_command_builds_n_ranks():
    b = load_bench()
    cmd = b.launcher_cmd(["--gpus", "8", "--steps", "512"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "512"] and cmd[-5] == BENCH


def test_launcher_parent_makes_no_gpu_call():
    """`bench.py --gpus 4` with WORLD_SIZE unset: the parent process (dry run: no PMC child,
    no CPU baseline, no ranks) builds the 4-rank command and has not initialised torch.cuda."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-dry-run", "--no-pmc", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["cuda_initialized"] is False
    assert "--nproc-per-node=4" in line["cmd"]
    assert line["cmd"][line["cmd"].index("--master-addr") + 1] == "127.0.0.1"
    assert not os.path.exists(line["parent_results"])  # the launcher cleans up its hand-off file


def test_parent_results_are_merged_by_the_ranks(tmp_path, monkeypatch):
    b = load_bench()
    p = tmp_path / "parent.json"
    p.write_text(json.dumps(dict(pmc=123.0, pmc_counters={"FETCH_SIZE": 1.0}, cpu_baseline={"value": 5.0})))
    monkeypatch.setenv("BENCH_PARENT_RESULTS", str(p))
    assert b.parent_results()["cpu_baseline"]["value"] == 5.0
    monkeypatch.setenv("BENCH_PARENT_RESULTS", str(tmp_path / "missing.json"))
    assert b.parent_results() is None


# ------------------------------------------------------------------ the gathered payload
N_TOTAL, T, STEPS = 48, 7, 40
KW = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002, slippage_bps=1.0)
GEN = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=T, seed=9)


def shard_summaries(n, offset, acts):
    """What he_episode_summaries holds for envs [offset, offset + n) after STEPS steps:
    the last finished episode's {return, sum step P&L, sum costs, length} (oracle sums)."""
    env = OracleVecEnv(n, mode="gbm", gen=dict(GEN, env_offset=offset), **KW)
    env.seed_envs_at(np.arange(n), [GEN["seed"]] * n)
    env.reset()
    run = np.zeros((3, n))
    length = np.zeros(n)
    last = np.zeros((n, 4))
    for s in range(STEPS):
        _, r, term, _, info = env.step(acts[s])
        run += np.stack([r, info["step_pnl_total"], info["transaction_costs_total"]])
        length += 1
        done = np.asarray(term, bool)
        last[done] = np.stack([run[0], run[1], run[2], length], 1)[done]
        run[:, done] = 0.0
        length[done] = 0
    return last.astype(np.float32)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = load_bench()
    n = N_TOTAL // world
    acts = np.random.default_rng(3).uniform(-1.05, 1.05, size=(STEPS, N_TOTAL, 2)).astype(np.float32)
    local = torch.from_numpy(shard_summaries(n, rank * n, acts[:, rank * n:(rank + 1) * n]))
    gathered = torch.empty((world * n, 4), dtype=torch.float32)
    b.gather_summaries(dist, local, gathered)
    if rank == 0:
        q.put((gathered.numpy(), b.summarize_payload(gathered)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_summary_gather_equals_one_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, stats = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    acts = np.random.default_rng(3).uniform(-1.05, 1.05, size=(STEPS, N_TOTAL, 2)).astype(np.float32)
    one = shard_summaries(N_TOTAL, 0, acts)
    assert np.array_equal(got, one)
    assert (one[:, 3] == T).all()  # every env finished STEPS // T episodes of length T
    assert stats["envs"] == N_TOTAL and stats["envs_with_finished_episode"] == N_TOTAL
    assert stats["mean_length"] == pytest.approx(T)


def _shard_check_worker(rank, world, port, q, corrupt):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = load_bench()
    n = N_TOTAL // world
    acts = np.random.default_rng(3).uniform(-1.05, 1.05, size=(STEPS, N_TOTAL, 2)).astype(np.float32)
    local = torch.from_numpy(shard_summaries(n, rank * n, acts[:, rank * n:(rank + 1) * n]))
    gathered = torch.empty((world * n, 4), dtype=torch.float32)
    b.gather_summaries(dist, local, gathered)
    # the neighbour's last 8 envs, re-run in a shard of their own at their global env ids
    nb, j0, m = b.shard_check_slice(rank, world, n, 8)
    assert (nb, j0, m) == ((rank + 1) % world, n - 8, 8)
    lo = nb * n + j0
    got = torch.from_numpy(shard_summaries(m, lo, acts[:, lo:lo + m]))
    if corrupt and rank == 1:
        got.view(torch.int32)[3, 1] ^= 1   # one bit of one env's P&L sum
    q.put((rank, b.shard_check_verdict(dist, got, gathered, nb, j0, n)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_two_rank_gloo_shard_check(corrupt):
    """the self-verifying N-rank line.  Each rank re-runs its neighbour's
    last envs in a shard of their own and compares the bits of their episode summaries with
    the all-gathered rows; every rank reports the combined verdict (one flipped bit on one
    rank -> MISMATCH everywhere, one mismatched row)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_check_worker, args=(r, 2, port, q, corrupt)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        v = res[r]
        assert v["ranks"] == 2 and v["envs_per_rank"] == 8
        if corrupt:
            assert v["result"] == "MISMATCH" and v["mismatched_rows"] == 1
        else:
            assert v["result"] == "bit-identical" and v["mismatched_rows"] == 0
            assert v["finished_episodes_in_checked_rows"] == 8


# ------------------------------------------------------------------ failing fast
def _selftest(extra_env, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(BENCH_DIST_BACKEND="gloo", **extra_env)
    import time
    t0 = time.time()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-selftest", "--no-pmc", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)
    return out, time.time() - t0


def test_two_rank_launch_completes_and_records_phases():
    out, _ = _selftest(dict(BENCH_DIST_TIMEOUT="60"))
    assert out.returncode == 0, out.stderr[-2000:]
    for r in (0, 1):
        assert f"[bench rank {r}/2] ready" in out.stderr and f"[bench rank {r}/2] done" in out.stderr


def test_rank_that_never_joins_fails_fast_and_is_named():
    """Rank 1 never calls init_process_group: rank 0's rendezvous times out after
    BENCH_DIST_TIMEOUT (not the driver's wall limit), the launcher exits non-zero and names
    rank 1 as not done, with its last phase."""
    out, took = _selftest(dict(BENCH_DIST_TIMEOUT="8", BENCH_TEST_STALL_RANK="1"))
    assert out.returncode != 0
    assert took < 120, took
    assert "ranks not done: [0, 1]" in out.stderr or "ranks not done: [1]" in out.stderr, out.stderr[-3000:]
    assert "rank 1: last phase: stalling" in out.stderr
    rep = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert 1 in rep["ranks_not_done"] and rep["last_phase"]["1"].startswith("stalling")


def test_launch_wall_limit_kills_the_child_group():
    """A child that outlives BENCH_LAUNCH_TIMEOUT is killed as a process group (rc 124) and
    the stalled rank is named."""
    out, took = _selftest(dict(BENCH_DIST_TIMEOUT="600", BENCH_TEST_STALL_RANK="1", BENCH_LAUNCH_TIMEOUT="15"))
    assert out.returncode == 124, (out.returncode, out.stderr[-2000:])
    assert took < 90, took
    assert "wall limit 15 s" in out.stderr and "rank 1: last phase: stalling" in out.stderr
