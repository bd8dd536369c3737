"""Multi-GPU plumbing: one process per GPU, envs sharded by global id.

Envs are independent, so a step needs no collective.  Each rank owns the
contiguous global ids [rank*N, (rank+1)*N) (he_config.global_env_offset); the
Philox subsequence of an env is its global id, so every trajectory is identical
for any GPU count.  Ranks exchange data only at rollout-buffer boundaries
(n_steps = 256 in train_ppo_v2.py:48): `gather_rollout` all-gathers per-env
tensors over RCCL (backend "nccl") on MI355X / gloo on CPU.
"""
import os

import torch


def world_info():
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard_offset(n_per_rank, rank):
    """Global id of this rank's first env (weak scaling: n_per_rank envs per GPU)."""
    if n_per_rank < 1 or rank < 0:
        raise ValueError("n_per_rank >= 1 and rank >= 0 required")
    return n_per_rank * rank


def init(backend=None, force=False, timeout_s=120.0):
    """Initialise the default process group for this process's device (at world size 1
    only with force=True: a one-rank group, e.g. to exercise RCCL on a one-GPU box).
    timeout_s bounds the rendezvous and every collective: a rank that never joins fails
    the others within it instead of hanging the job."""
    import datetime
    import torch.distributed as dist
    rank, local, world = world_info()
    if dist.is_initialized() or (world == 1 and not force):
        return rank, local, world
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    timeout = datetime.timedelta(seconds=float(timeout_s))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local), timeout=timeout)
    else:
        dist.init_process_group(backend, timeout=timeout)
    return rank, local, world


def gather_rollout(t, group=None, env_dim=0):
    """All-gather a per-env tensor from every rank in global-id order (rank r's envs are the
    global ids [r N, (r + 1) N), shard_offset).

    env_dim = 0: [N, ...] -> [world * N, ...] (per-env records: episode summaries).
    env_dim = 1: [K, N, ...] -> [K, world * N, ...] (he_rollout's obs / reward / terminated,
    step-major): the collective concatenates the ranks' [K, N, ...] blocks rank-major, so the
    result is [world, K, N, ...] re-laid out as [K, world, N, ...] (one device copy) --
    SURVEY 8(e)'s rollout-tensor gather at the buffer boundary (train_ppo_v2.py:48), for
    small N only (config 4's full tensors are ~9 GB per rank)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return t
    if env_dim not in (0, 1) or t.dim() <= env_dim:
        raise ValueError("env_dim must be 0 or 1 and a dimension of t")
    w = dist.get_world_size(group)
    t = t.contiguous()
    out = torch.empty((w * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    if env_dim == 0 or w == 1:
        return out
    k, n = t.shape[0], t.shape[1]
    rest = tuple(t.shape[2:])
    return out.view((w, k, n) + rest).transpose(0, 1).reshape((k, w * n) + rest)
