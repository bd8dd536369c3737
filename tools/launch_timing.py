#!/usr/bin/env python3
"""Where the timed region's per-launch time goes: back-to-back he_rollout launches of a
bench config timed three ways on the launching stream --
  probe   he_time_next_step: HIP events inside the dispatch (hipExtLaunchKernelGGL)
  marker  hipEventRecord between consecutive launches (kernel + the gap before the next)
  region  one pair of events around the whole sequence / launches
-- so the gap between dispatches and any slow-down of sustained runs show separately.

    python tools/launch_timing.py [--config 2] [--launches 30]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--k", type=int, default=256)
    args = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[args.config]
    a = bench.parse(["--config", str(args.config), "--rollout-k", str(args.k)])
    a.envs = cfg["envs"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    env = bench.make_env(a, dev)
    n = a.envs
    acts = torch.rand((args.k, n, 2), device=dev) * 2 - 1
    obs = torch.empty((args.k, n, 13), device=dev)
    rew = torch.empty((args.k, n), device=dev)
    term = torch.empty((args.k, n), dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(device=dev)
    lib, h = env.lib, env._h
    hev = bench.HipEvents()

    def launch():
        if lib.he_rollout(h, args.k, acts.data_ptr(), obs.data_ptr(), rew.data_ptr(), term.data_ptr(),
                          st.cuda_stream):
            raise RuntimeError(lib.he_last_error(h).decode())

    with torch.cuda.stream(st):
        for _ in range(5):
            launch()
    torch.cuda.synchronize()
    out = {}
    L = args.launches
    # probe: events inside each dispatch, plus one region around all of them
    kev = [(hev.create(), hev.create()) for _ in range(L)]
    r0, r1 = hev.create(), hev.create()
    with torch.cuda.stream(st):
        hev.record(r0, st)
        for k in range(L):
            lib.he_time_next_step(h, kev[k][0], kev[k][1])
            launch()
        hev.record(r1, st)
    torch.cuda.synchronize()
    probe = np.array([hev.elapsed_ms(x, y) for x, y in kev]) * 1e3
    gaps = np.array([hev.elapsed_ms(kev[k][1], kev[k + 1][0]) for k in range(L - 1)]) * 1e3
    out["probe_us"] = dict(mean=float(probe.mean()), min=float(probe.min()), max=float(probe.max()),
                           first5=[round(x, 1) for x in probe[:5]], last5=[round(x, 1) for x in probe[-5:]])
    out["gap_us_between_probed_dispatches"] = dict(mean=float(gaps.mean()), max=float(gaps.max()))
    out["region_with_probes_us_per_launch"] = hev.elapsed_ms(r0, r1) * 1e3 / L
    # markers: plain hipEventRecord between plain launches
    mev = [hev.create() for _ in range(L + 1)]
    with torch.cuda.stream(st):
        hev.record(mev[0], st)
        for k in range(L):
            launch()
            hev.record(mev[k + 1], st)
    torch.cuda.synchronize()
    mk = np.array([hev.elapsed_ms(mev[k], mev[k + 1]) for k in range(L)]) * 1e3
    out["marker_us"] = dict(mean=float(mk.mean()), min=float(mk.min()), max=float(mk.max()),
                            first5=[round(x, 1) for x in mk[:5]], last5=[round(x, 1) for x in mk[-5:]])
    # region only
    with torch.cuda.stream(st):
        hev.record(r0, st)
        for k in range(L):
            launch()
        hev.record(r1, st)
    torch.cuda.synchronize()
    out["region_us_per_launch"] = hev.elapsed_ms(r0, r1) * 1e3 / L
    out.update(config=args.config, envs=n, k=args.k, launches=L)
    print(json.dumps(out, indent=1))
    env.close()


if __name__ == "__main__":
    main()
