#!/usr/bin/env python3
"""Where lds_rollout_kernel's wave roles land: per CU, which SIMD hosts which role.

Needs a -DHE_LDS_HWID build (tools/ab/hwid.so, or a -DHE_LDS_HWID -DHE_LDS_BALANCE=1
one): every wave records {HW_ID, XCC_ID, per-CU ticket, role}.  Runs one 256-step
rollout at the bench config's env count and prints the placement statistics:
workgroups per CU, whether a workgroup's 4 waves sit on 4 distinct SIMDs, and how many
waves of each role the busiest SIMD of a CU carries.

    CANTORRL_HEDGEENV_LIB=tools/ab/hwid.so python tools/lds_hwid.py [--config 2]
"""
import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ROLES = ("reward", "obs", "prod0", "prod1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--k", type=int, default=256)
    args = ap.parse_args()
    import bench
    from cantorrl_amd.vec_env import HedgingVecEnv
    cfg = bench.CONFIGS[args.config]
    n = cfg["envs"]
    env = HedgingVecEnv(n, mode=cfg["mode"], generate=cfg["gen"], seed=42, return_numpy=False, info_keys=(),
                        **cfg["kw"])
    env.reset_tensors()
    acts = torch.rand((args.k, n, 2), device="cuda") * 2 - 1
    env.rollout(acts)
    torch.cuda.synchronize()
    lib = env.lib
    nwg = (n + 63) // 64
    buf = np.zeros((16384, 4, 4), np.uint32)
    lib.he_debug_lds_hwid.restype = ctypes.c_int32
    lib.he_debug_lds_hwid.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.he_debug_lds_hwid(buf.ctypes.data, buf.nbytes) == 0
    env.close()
    rec = buf[:min(nwg, 16384)]
    hw, xcc, ticket, rolem = rec[..., 0], rec[..., 1], rec[..., 2], rec[..., 3]
    simd = (hw >> 4) & 3
    cu = ((xcc & 15) << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    role = rolem & 0xFF
    distinct = ((rolem >> 8) & 0xFF) == 15
    wg_cu = cu[:, 0]
    same_cu = (cu == wg_cu[:, None]).all(1)
    per_cu = collections.Counter(wg_cu.tolist())
    # per CU: role counts per SIMD over its workgroups
    load = collections.defaultdict(lambda: np.zeros((4, 4), np.int64))  # [simd][role]
    for w in range(rec.shape[0]):
        for v in range(4):
            load[int(wg_cu[w])][int(simd[w, v]), int(role[w, v])] += 1
    max_obs = collections.Counter(int(m[:, 1].max()) for m in load.values())
    max_role = {ROLES[r]: dict(collections.Counter(int(m[:, r].max()) for m in load.values())) for r in range(4)}
    start = collections.Counter(int(simd[w, 0]) for w in range(rec.shape[0]))
    order = collections.Counter(tuple(int(x) for x in simd[w]) for w in range(rec.shape[0]))
    out = dict(config=args.config, envs=n, workgroups=int(rec.shape[0]), cus=len(per_cu),
               wg_per_cu=dict(collections.Counter(per_cu.values())),
               waves_on_one_cu=bool(same_cu.all()), distinct_simds=float(distinct[:, 0].mean()),
               wave0_simd=dict(start), simd_orders=dict((str(k), v) for k, v in order.most_common(8)),
               max_obs_waves_per_simd=dict(max_obs), max_waves_per_simd_by_role=max_role,
               xcc_values=sorted(set(int(x) for x in np.unique(xcc & 15))))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
