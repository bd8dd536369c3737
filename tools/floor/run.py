#!/usr/bin/env python3
"""Launch floors of the Gym-API step path: floor_empty / floor_copy (tools/floor/floor.hip)
at he_step's grid, 64 launches per hipGraph as bench.py --mode graph replays he_step, and
the real step1_kernel beside them; HIP-event time per launch over 20 graph replays.

    python tools/floor/run.py build        (CPU: hipcc -> tools/floor/libfloor.so)
    python tools/floor/run.py [--envs 65536]
Run under rocprofv3 --kernel-trace --stats for each kernel's own average duration.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SO = os.path.join(HERE, "libfloor.so")


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                    os.path.join(HERE, "floor.hip")], check=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    args = ap.parse_args()
    import torch
    sys.path.insert(0, REPO)
    import bench
    n = args.envs
    lib = ctypes.CDLL(SO)
    lib.floor_launch.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    inp = torch.rand((4 * n * 4,), device=dev)
    out = torch.zeros((n * 19,), device=dev)
    st = torch.cuda.Stream(device=dev)
    res = {}
    for which, name in ((0, "floor_empty"), (1, "floor_copy")):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            lib.floor_launch(which, n, inp.data_ptr(), out.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                for _ in range(64):
                    lib.floor_launch(which, n, inp.data_ptr(), out.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record(st)
            for _ in range(20):
                g.replay()
            e1.record(st)
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1e3 / (20 * 64), 3)
    # the real he_step in the bench's graph mode (64 launches per graph + the market block)
    a = bench.parse(["--mode", "graph"])
    a.envs = n
    env = bench.make_env(a, dev)
    acts = torch.rand((256, n, 2), device=dev) * 2 - 1
    r = bench.Runner(a, env, "graph", acts, st)
    wall, dev_ms = bench.timed(r, 20 * 64, 4 * 64, None)
    res["he_step_graph_us_per_step"] = round(dev_ms * 1e3 / (20 * 64), 3)
    env.close()
    res["envs"] = n
    print(json.dumps(res))


if __name__ == "__main__":
    main()
