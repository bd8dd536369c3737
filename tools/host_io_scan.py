"""HedgingVecEnv.step_async + step_wait (NumPy in, NumPy out, Monitor on) with the host-mapped
block (host_io=True: the kernel reads the actions from and writes obs / reward / flags / infos
into pinned host memory, the completion word raised after them) against the device io buffer + one
pinned DMA (host_io=False), by env count: where HOST_IO_MAX_ENVS should sit.

    python tools/host_io_scan.py [n1,n2,...] [steps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cantorrl_amd.vec_env import HedgingVecEnv, MONITOR_KEYWORDS  # noqa: E402


def main():
    ns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,256,4096,8192,16384,65536").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    torch.cuda.set_device(0)
    for n in ns:
        row = [f"n {n:6d}"]
        for hio in (True, False):
            env = HedgingVecEnv(n, mode="gbm", generate=bench.GEN, seed=42, monitor_keywords=MONITOR_KEYWORDS,
                                host_io=hio, **bench.TRAIN_KW)
            env.reset()
            rng = np.random.default_rng(0)
            acts = [rng.uniform(-1, 1, size=(n, 2)).astype(np.float32) for _ in range(8)]
            for k in range(30):
                env.step_async(acts[k % 8])
                env.step_wait()
            ts = np.empty(steps)
            for k in range(steps):
                t0 = time.perf_counter()
                env.step_async(acts[k % 8])
                env.step_wait()
                ts[k] = time.perf_counter() - t0
            env.close()
            row.append(f"host_io={hio!s:5s} median {np.median(ts) * 1e6:9.1f} us  mean {ts.mean() * 1e6:9.1f} us")
        print("   ".join(row), flush=True)


if __name__ == "__main__":
    main()
