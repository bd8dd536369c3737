"""Device time of the auxiliary kernels: DeviceVecNormalize per step at 65,536 envs
(he_vecnorm_step: moments + apply) and the path analytics at 1M paths x 253 columns."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cantorrl_amd import _lib, analytics as an  # noqa: E402
from cantorrl_amd.vec_env import HedgingVecEnv  # noqa: E402
from cantorrl_amd.vec_normalize import DeviceVecNormalize  # noqa: E402

dev = "cuda:0"
KW = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002, slippage_bps=1.0)
GEN = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=252)


def ev():
    return torch.cuda.Event(enable_timing=True)


n = 65536
env = HedgingVecEnv(n, mode="gbm", generate=GEN, seed=1, device=dev, return_numpy=False, info_keys=(), **KW)
vn = DeviceVecNormalize(env)
vn.reset_tensors()
acts = torch.rand((64, n, 2), device=dev) * 2 - 1
for k in range(16):
    vn.step_tensors(acts[k])
torch.cuda.synchronize()
lib = env.lib
p = vn._params()
P = vn._p
args = [ctypes.byref(p), n, P(env._obs), P(env._rew), P(env._term), P(env._tobs), P(vn._returns), P(vn._stats),
        P(vn._scratch), P(vn._obs_out), P(vn._rew_out), P(vn._tobs_out), P(vn._ep_ret), P(vn._ep_len),
        P(vn._ep_ret_done), P(vn._ep_len_done), vn._stream()]
e0, e1 = ev(), ev()
e0.record()
R = 200
for _ in range(R):
    lib.he_vecnorm_step(*args)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / R
print(f"he_vecnorm_step n={n}: {us:.2f} us/step (statistics update + normalize), {n * 68 / (us * 1e-6) / 1e9:.1f} GB/s "
      f"of obs+reward in/out", flush=True)
# frozen statistics (eval): the normalize phase alone, no cross-workgroup merge
p.training = 0
e0.record()
for _ in range(R):
    lib.he_vecnorm_step(*args)
e1.record()
torch.cuda.synchronize()
print(f"he_vecnorm_step n={n}, training=False: {e0.elapsed_time(e1) * 1e3 / R:.2f} us/step", flush=True)
p.training = 1
# the second half alone (he_vecnorm_apply): what a step costs on top of he_step when the
# moments run inside he_step's launch (he_vecnorm_attach)
e0.record()
for _ in range(R):
    lib.he_vecnorm_apply(*args)
e1.record()
torch.cuda.synchronize()
print(f"he_vecnorm_apply n={n} (statistics update + normalize; moments fused into he_step): "
      f"{e0.elapsed_time(e1) * 1e3 / R:.2f} us/step", flush=True)
# env step + vecnorm, eager (one Python call per step, as SB3 drives it): device time per step
# between two events, and the host's wall time per call over 256 calls (an eager loop is
# host-issue-bound when the latter is the larger)


def eager_us(step, label, steps=256):
    for k in range(8):
        step(k)
    torch.cuda.synchronize()
    e0.record()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k % 64)
    wall = (time.perf_counter() - t0) * 1e6 / steps
    e1.record()
    torch.cuda.synchronize()
    dev_us = e0.elapsed_time(e1) * 1e3 / steps
    print(f"eager, {label}: {dev_us:.2f} us/step device (events), {wall:.2f} us/step host wall per call", flush=True)
    return dev_us, wall


eager_us(lambda k: vn.step_tensors(acts[k]), "env he_step + vecnorm, moments fused into he_step")
vn._fusable = False  # detach: he_step, then he_vecnorm_step (moments + apply)
eager_us(lambda k: vn.step_tensors(acts[k]), "env he_step + vecnorm, separate moments launch")
vn._fusable = True
vn.training = False
eager_us(lambda k: vn.step_tensors(acts[k]), "env he_step + vecnorm eval (fused into he_step)")
vn.training = True
eager_us(lambda k: env.step_tensors(acts[k]), "env he_step alone")


def graph_us(step, label, reps=20):
    """Device time per step of 64 steps captured into one hipGraph (the bench's graph mode:
    one market block per graph, so market_kernel is amortised over its 64 steps), replayed
    `reps` times between two events on the capture stream."""
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        for k in range(64):   # one eager block: the captured block starts at a block boundary
            step(k)
        env.sync_market()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for k in range(64):
            step(k)
        env.sync_market()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = ev(), ev()
    with torch.cuda.stream(s):
        a.record(s)
        for _ in range(reps):
            g.replay()
        b.record(s)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / (64 * reps)
    print(f"graph mode, {label}: {us:.2f} us/step (64 steps per graph incl. the block's market_kernel)", flush=True)
    return us


graph_us(lambda k: env.step_tensors(acts[k]), "he_step alone")
vn._fusable = True
graph_us(lambda k: vn.step_tensors(acts[k]), "he_step + VecNormalize, moments fused into he_step")
vn._fusable = False
graph_us(lambda k: vn.step_tensors(acts[k]), "he_step + VecNormalize, separate moments launch")
vn.training = False
vn._fusable_eval = False
graph_us(lambda k: vn.step_tensors(acts[k]), "he_step + VecNormalize, frozen statistics (eval), he_vecnorm_step launch")
vn._fusable_eval = True
graph_us(lambda k: vn.step_tensors(acts[k]), "he_step + VecNormalize, frozen statistics (eval), fused into he_step")
vn.training = True
env.close()

g = torch.Generator(device=dev).manual_seed(0)
N, T1 = 1 << 20, 253
inc = torch.randn((N, T1), generator=g, device=dev, dtype=torch.float64) * 0.01
inc[:, 0] = 0
paths = 100 * torch.exp(torch.cumsum(inc, dim=1))
del inc
an.fixed_european_marks(paths, device=dev)
an.bs_delta_hedge(paths, device=dev)
torch.cuda.synchronize()
for name, fn in (("he_fixed_european_marks", lambda: an.fixed_european_marks(paths, device=dev)),
                 ("he_bs_delta_hedge", lambda: an.bs_delta_hedge(paths, device=dev))):
    e0.record()
    for _ in range(3):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    el = N * T1
    print(f"{name} {N} paths x {T1}: {ms:.2f} ms  {el / (ms * 1e-3):.3g} path-columns/s", flush=True)
    del out
