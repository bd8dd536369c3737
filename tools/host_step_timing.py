"""Where the single-env / N_ENVS=2 host step spends its time (MI355X): the raw he_step + he_stream_wait
through the host-mapped block, HedgingVecEnv.step_host, HedgingEnv.step, and the baselines.py-shaped
loop's policy alone.

    python tools/host_step_timing.py
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cantorrl_amd.env import HedgingEnv  # noqa: E402


def med(fn, n=3000, warm=200):
    for _ in range(warm):
        fn()
    ts = np.empty(n)
    for i in range(n):
        a = time.perf_counter()
        fn()
        ts[i] = time.perf_counter() - a
    return round(float(np.median(ts)) * 1e6, 2), round(float(ts.mean()) * 1e6, 2)


def main():
    torch.cuda.set_device(0)
    env = HedgingEnv(mode="gbm", generate=bench.GEN, **bench.TRAIN_KW)
    env.reset()
    v = env._venv
    z = v._hio
    lib = v.lib
    st = torch.cuda.current_stream().cuda_stream
    act = np.array([0.1, -0.2], np.float32)
    out = {}

    def raw():   # (no autoreset on this handle: past T the env stays terminated, same work)
        lib.he_step(v._h, *z.step_args, st)
        lib.he_stream_wait(st)
    out["he_step+he_stream_wait"] = med(raw)

    def raw_sig():   # the kernel raises the block's flag word (he_step_signal), the host reads it
        lib.he_step_signal(v._h, z.d_flag)
        lib.he_step(v._h, *z.step_args, st)
        lib.he_signal_wait(v._h, z.h_flag, st)
    out["he_step_signal+he_step+he_signal_wait"] = med(raw_sig)

    def launch_only():
        lib.he_step(v._h, *z.step_args, st)
    out["he_step launch only (no wait)"] = med(launch_only, 2000, 100)
    torch.cuda.synchronize()
    # the same step with device-resident buffers (no host-mapped reads / writes in the kernel)
    dev_args = (v._act.data_ptr(), v._obs.data_ptr(), v._rew.data_ptr(), v._term.data_ptr(), v._trunc.data_ptr(),
                v._tobs.data_ptr(), z.step_args[-1])

    def raw_dev():
        lib.he_step(v._h, *dev_args, st)
        lib.he_stream_wait(st)
    out["he_step (device buffers)+he_stream_wait"] = med(raw_dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
    hip.hipStreamQuery.restype = ctypes.c_int

    def raw_spin():   # completion by polling hipStreamQuery instead of a blocking synchronize
        lib.he_step(v._h, *z.step_args, st)
        while hip.hipStreamQuery(st) != 0:
            pass
    out["he_step+poll hipStreamQuery"] = med(raw_spin)

    def empty_sync():
        lib.he_stream_wait(st)
    out["he_stream_wait on an idle stream"] = med(empty_sync)
    out["step_host"] = med(lambda: v.step_host(act))
    env.reset()

    def step():
        if env._terminated:
            env.reset()
        return env.step(act)
    out["HedgingEnv.step (+ a reset every 252)"] = med(step)
    obs = step()[0]

    def policy():
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
    out["policy_delta_every_step (caller's)"] = med(policy)
    ev = torch.cuda.Event()
    out["torch Event record+synchronize (empty)"] = med(lambda: (ev.record(), ev.synchronize()))
    env.close()
    for k, (m, a) in out.items():
        print(f"{k:45s} median {m:8.2f} us  mean {a:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
