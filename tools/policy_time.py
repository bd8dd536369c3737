"""Device time of he_rollout_policy (the baseline policies fused into the rollout, baselines.py:74-103,
delta_and_nothing.py:122-163) at the headline's env count, against he_rollout with stored actions.

    python tools/policy_time.py [n_envs] [K] [launches] [gbm|gbm_v1|replay]

replay: the baselines' own setting (baselines.py:132-138: the v1 env on an NPZ of paths), here a
synthetic 100,000 x 253 table (bench.replay_tables).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cantorrl_amd.vec_env import HedgingVecEnv  # noqa: E402


def timed(fn, launches):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(launches):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / launches * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    mode = sys.argv[4] if len(sys.argv) > 4 else "gbm"
    if mode == "gbm_v1":   # a configuration outside the lean one: the generic LDS steppers
        env = HedgingVecEnv(n, mode="gbm", generate=bench.GEN, variant=1, seed=42, return_numpy=False,
                            info_keys=())
    elif mode == "replay":
        env = HedgingVecEnv(n, tables=bench.replay_tables(paths=100000, cols=253), variant=1, seed=42,
                            return_numpy=False, info_keys=())
    else:
        env = HedgingVecEnv(n, mode="gbm", generate=bench.GEN, seed=42, return_numpy=False, info_keys=(),
                            **bench.TRAIN_KW)
    print(f"mode {mode}, {n} envs, K = {K}, {L} launches", flush=True)
    env.reset_tensors()
    acts = torch.rand((K, n, 2), device="cuda") * 2 - 1
    obs = torch.empty((K, n, 13), device="cuda")
    rew = torch.empty((K, n), device="cuda")
    term = torch.empty((K, n), dtype=torch.uint8, device="cuda")
    us = timed(lambda: env.rollout(acts, obs, rew, term), L)
    print(f"he_rollout (stored actions)       {us:9.1f} us per launch  {n * K / us * 1e6:.3e} env-steps/s", flush=True)
    for pol in ("no_hedge", "delta_every_step", "delta_threshold"):
        us = timed(lambda: env.rollout_policy(K, pol, obs=obs, reward=rew, terminated=term), L)
        print(f"he_rollout_policy {pol:16s} {us:9.1f} us per launch  {n * K / us * 1e6:.3e} env-steps/s", flush=True)
    env.close()


if __name__ == "__main__":
    main()
