"""world_size-2 gloo test of the N>1 path on CPU: each rank steps its shard of
envs (global ids offset by rank, as bench.py does on MI355X), ranks all-gather the
per-env results at the rollout boundary, and the gathered rollout equals one
process stepping every env -- the Philox keying makes trajectories independent of
the shard count."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle.hedging_oracle import OracleVecEnv

N_TOTAL, STEPS, T = 64, 30, 12
KW = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002, slippage_bps=1.0)
GEN = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=T, seed=5)


def run_shard(n, offset, acts):
    env = OracleVecEnv(n, mode="gbm", gen=dict(GEN, env_offset=offset), **KW)
    env.seed_envs_at(np.arange(n), [GEN["seed"]] * n)
    env.reset()
    rew, obs = [], []
    for s in range(STEPS):
        o, r, term, _, _ = env.step(acts[s])
        rew.append(r)
        obs.append(o)
    return np.stack(rew, 1), np.stack(obs, 1)  # [n, STEPS], [n, STEPS, 13]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from cantorrl_amd import dist as hd
    import torch.distributed as dist
    hd.init(backend="gloo")
    n = N_TOTAL // world
    off = hd.shard_offset(n, rank)
    acts = np.random.default_rng(1).uniform(-1, 1, size=(STEPS, N_TOTAL, 2)).astype(np.float32)
    rew, obs = run_shard(n, off, acts[:, off:off + n])
    g_rew = hd.gather_rollout(torch.from_numpy(rew))
    g_obs = hd.gather_rollout(torch.from_numpy(obs))
    # he_rollout's step-major layout [K, N, ...] gathered along the env dimension
    k_rew = hd.gather_rollout(torch.from_numpy(np.ascontiguousarray(rew.T)), env_dim=1)
    k_obs = hd.gather_rollout(torch.from_numpy(np.ascontiguousarray(obs.transpose(1, 0, 2))), env_dim=1)
    if rank == 0:
        q.put((g_rew.numpy(), g_obs.numpy(), k_rew.numpy(), k_obs.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_shards_equal_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g_rew, g_obs, k_rew, k_obs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    acts = np.random.default_rng(1).uniform(-1, 1, size=(STEPS, N_TOTAL, 2)).astype(np.float32)
    rew, obs = run_shard(N_TOTAL, 0, acts)
    assert np.array_equal(g_rew, rew)
    assert np.array_equal(g_obs, obs)
    # [K, world * N, ...] in global env order: the single process's step-major tensors
    assert k_rew.shape == (STEPS, N_TOTAL) and k_obs.shape == (STEPS, N_TOTAL, 13)
    assert np.array_equal(k_rew, rew.T)
    assert np.array_equal(k_obs, obs.transpose(1, 0, 2))


def test_gather_rollout_env_dim_checks():
    from cantorrl_amd import dist as hd
    t = torch.zeros(3)
    assert hd.gather_rollout(t, env_dim=1) is t   # no process group: the local tensor
    import torch.distributed as dist
    assert not dist.is_initialized()


def test_shard_offset_contract():
    from cantorrl_amd import dist as hd
    assert [hd.shard_offset(65536, r) for r in range(4)] == [0, 65536, 131072, 196608]
    with pytest.raises(ValueError):
        hd.shard_offset(0, 1)
