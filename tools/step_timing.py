#!/usr/bin/env python3
"""Where the time of one he_step (step1_kernel) goes, per wave (diagnostic build -DHE_TIMING):

    CANTORRL_HEDGEENV_LIB=tools/abt/steptim.so python tools/step_timing.py [n_envs]

Points (step_body HE_TIM): 0 kernel entry, 1 after the Params copy, 2 after the prologue
loads, 3 before the obs flush, 4 end.  Prints, over the last launch's waves, the spread of
entry / exit times (100 MHz s_memrealtime, relative to the first entry) and the median /
p90 shader cycles between points."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cantorrl_amd.vec_env import HedgingVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cfg = bench.CONFIGS[2]
env = HedgingVecEnv(n, mode="gbm", generate=cfg["gen"], seed=42, return_numpy=False, info_keys=(), **cfg["kw"])
env.reset_tensors()
acts = torch.rand((n, 2), device="cuda") * 2 - 1
for _ in range(70):
    env.step_tensors(acts, terminal_obs=False)
torch.cuda.synchronize()
for _ in range(3):
    env.step_tensors(acts, terminal_obs=False)  # the last launch is within a market block
torch.cuda.synchronize()
lib = env.lib
lib.he_debug_timing.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros((5, 8192, 2), np.uint64)
assert lib.he_debug_timing(buf.ctypes.data, buf.nbytes) == 0
waves = (n + 63) // 64
b = buf[:, :waves, :].astype(np.int64)
rt0, rt4 = b[0, :, 0], b[4, :, 0]
t0 = rt0.min()
print("waves", waves)
print("entry (10 ns ticks after the first): p0 %d p50 %d p90 %d max %d" % tuple(np.percentile(rt0 - t0, [0, 50, 90, 100])))
print("exit  (10 ns ticks after the first entry): p0 %d p50 %d p90 %d max %d" % tuple(np.percentile(rt4 - t0, [0, 50, 90, 100])))
for a, c in ((0, 1), (1, 2), (2, 3), (3, 4), (0, 4)):
    d = b[c, :, 1] - b[a, :, 1]
    print("cycles %d->%d: p10 %d p50 %d p90 %d" % ((a, c) + tuple(np.percentile(d, [10, 50, 90]))))
env.close()
