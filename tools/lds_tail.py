#!/usr/bin/env python3
"""Why the last workgroups of lds_rollout_kernel finish late: per-workgroup wall time on the
100 MHz clock joined with where each workgroup ran (XCD, CU, SIMD of each role, its ticket).

Needs a -DHE_LDS_TIMING -DHE_LDS_HWID build (tools/abt/tail.so).  Runs a few 256-step
rollouts at a bench config's env count, saves the raw records of the last one to
<out>.npz and prints the wall-time distribution by XCD, by the workgroup's slot on its CU
(ticket mod 4), and for the slowest workgroups.

    CANTORRL_HEDGEENV_LIB=tools/abt/tail.so python tools/lds_tail.py [--config 2] [--out gpurun_out/tail]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "tail"))
    args = ap.parse_args()
    import bench
    from cantorrl_amd.vec_env import HedgingVecEnv
    cfg = bench.CONFIGS[args.config]
    n = cfg["envs"]
    env = HedgingVecEnv(n, mode=cfg["mode"], generate=cfg["gen"], seed=42, return_numpy=False, info_keys=(),
                        **cfg["kw"])
    env.reset_tensors()
    acts = torch.rand((args.k, n, 2), device="cuda") * 2 - 1
    for _ in range(6):
        env.rollout(acts)
    torch.cuda.synchronize()
    lib = env.lib
    nwg = min((n + 63) // 64, 4096)
    tim = np.zeros((4, 4096, 5), np.uint64)
    hwid = np.zeros((16384, 4, 4), np.uint32)
    for f, b in (("he_debug_lds_timing", tim), ("he_debug_lds_hwid", hwid)):
        fn = getattr(lib, f)
        fn.restype = ctypes.c_int32
        fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        assert fn(b.ctypes.data, b.nbytes) == 0, f
    env.close()
    tim, hwid = tim[:, :nwg], hwid[:nwg]
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    np.savez(args.out + ".npz", tim=tim, hwid=hwid)
    hw, xcc, ticket, rolem = hwid[..., 0], hwid[..., 1], hwid[..., 2], hwid[..., 3]
    simd = (hw >> 4) & 3
    cu = (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    role = rolem & 0xFF
    st = tim[:, :, 3].astype(np.float64).min(axis=0)
    en = tim[:, :, 4].astype(np.float64).max(axis=0)
    wall = (en - st) / 100.0
    t0 = st.min()
    x = xcc[:, 0] & 15
    slot = ticket[:, 0] & 3
    print(f"{nwg} workgroups: wall p50 {np.median(wall):.1f} p90 {np.percentile(wall, 90):.1f} max {wall.max():.1f} us; "
          f"first start -> last end {(en.max() - t0) / 100:.1f} us")
    for name, key in (("xcd", x), ("slot on CU (ticket mod 4)", slot)):
        print(f"by {name}:", " ".join(f"{k}:{np.median(wall[key == k]):.1f}/{wall[key == k].max():.1f}"
                                      for k in np.unique(key)))
    # per role: the SIMD it ran on and its busy cycles (not in barriers)
    busy = (tim[:, :, 0] - tim[:, :, 1]).astype(np.float64) / args.k
    order = np.argsort(wall)[::-1]
    print("slowest workgroups: wg xcd cu ticket wall | role->simd | busy/step per role")
    for g in order[:12]:
        rs = {int(role[g, w]): int(simd[g, w]) for w in range(4)}
        print(f"  {g:5d} {x[g]} {cu[g, 0]:3d} {ticket[g, 0]:6d} {wall[g]:6.1f} | "
              f"{[rs.get(r) for r in range(4)]} | {busy[:, g].round(0).tolist()}")
    # CUs: the spread of their workgroups' walls
    key = x.astype(np.int64) * 1024 + cu[:, 0]
    cus = np.unique(key)
    cu_max = np.array([wall[key == k].max() for k in cus])
    cu_min = np.array([wall[key == k].min() for k in cus])
    print(f"CUs {len(cus)}: max wall per CU p50 {np.median(cu_max):.1f} max {cu_max.max():.1f}; "
          f"in-CU spread (max - min) p50 {np.median(cu_max - cu_min):.1f} max {(cu_max - cu_min).max():.1f} us")


if __name__ == "__main__":
    main()
