#!/usr/bin/env python3
"""Per-role barrier waits of lds_rollout_kernel (diagnostic build -DHE_LDS_TIMING).

    CANTORRL_HEDGEENV_LIB=tools/abt/timing.so python tools/lds_timing.py [n_envs] [K] [bench config]

Roles: 0 reward stepper, 1 obs stepper, 2-3 producers (replay, config 6: the loaders).  For each: mean cycles from the
first barrier to the end and the share of them spent waiting in barriers (s_memtime), and the shader
clock over the same interval (s_memtime cycles per s_memrealtime tick, a 100 MHz counter).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cantorrl_amd.vec_env import HedgingVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 256
cfg = bench.CONFIGS[int(sys.argv[3]) if len(sys.argv) > 3 else 2]
if cfg["mode"] == "replay":  # lds_replay_kernel: roles 2-3 are the loader waves
    env = HedgingVecEnv(n, tables=bench.replay_tables(**cfg["table"]), seed=42, return_numpy=False, info_keys=(),
                        **cfg["kw"])
else:
    env = HedgingVecEnv(n, mode=cfg["mode"], generate=cfg["gen"], seed=42, return_numpy=False, info_keys=(),
                        **cfg["kw"])
env.reset_tensors()
acts = torch.rand((K, n, 2), device="cuda") * 2 - 1
for _ in range(4):
    env.rollout(acts)
torch.cuda.synchronize()
lib = env.lib
lib.he_debug_lds_timing.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros((4, 4096, 5), np.uint64)
assert lib.he_debug_lds_timing(buf.ctypes.data, buf.nbytes) == 0
wg = min((n + 63) // 64, 4096)
# the persistent grid (more tiles than resident workgroups): only blockIdx < grid hold records
# (each its last tile's); keep the filled rows
wg = int(min(wg, max(1, (buf[0, :, 2] > 0).sum())))
for role, name in enumerate(("reward", "obs", "prod0", "prod1")):
    tot = buf[role, :wg, 0].astype(np.float64)
    bar = buf[role, :wg, 1].astype(np.float64)
    print(f"{name:7s} total {tot.mean():12.0f} cyc  in barriers {bar.mean():12.0f} ({bar.mean() / tot.mean():6.1%})"
          f"  per step {tot.mean() / K:8.0f}  busy/step {(tot.mean() - bar.mean()) / K:8.0f}"
          f"  clock {tot.mean() * 100.0 / buf[role, :wg, 2].astype(np.float64).mean():6.0f} MHz"
          f"  wall {buf[role, :wg, 2].astype(np.float64).mean() / 100.0:8.1f} us")
# the launch's spread: every workgroup's start / end on the shared 100 MHz clock (roles 0-3)
st = buf[:, :wg, 3].astype(np.float64).min(axis=0)
en = buf[:, :wg, 4].astype(np.float64).max(axis=0)
t0 = st.min()
print(f"workgroups {wg}: start spread {(st.max() - t0) / 100:.1f} us (p50 {(np.median(st) - t0) / 100:.1f}), "
      f"end spread {(en.max() - en.min()) / 100:.1f} us, first start -> last end {(en.max() - t0) / 100:.1f} us, "
      f"workgroup wall p50 {np.median(en - st) / 100:.1f} / max {(en - st).max() / 100:.1f} us")
