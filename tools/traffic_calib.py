#!/usr/bin/env python3
"""Calibrate the gfx950 read-traffic counters on known byte counts, then read the step kernels'
traffic with the calibrated formula.

MI355X_MICROARCH.md ("HBM"): FETCH_SIZE reports 1/2 of a wide coalesced read on gfx950, and
other access widths are uncalibrated.  rocprofv3's FETCH_SIZE expression for gfx950 counts
TCC_BUBBLE as the 128-B requests; gfx950 also has per-size request counters
(TCC_EA0_RDREQ_{32B,64B,128B}) and a 32-B-unit count of the DRAM-bound reads
(TCC_EA0_RDREQ_DRAM_32B, "a 64-byte request counted as 2, 128-byte as 4").  This tool runs
three calibration kernels over a 1 GiB table (tools/calib/calib.hip: the wide coalesced
stream, the replay loaders' two 64-B half lines per row, a whole 128-B line per lane), then the headline rollout
(config 2) and the replay rollout (config 6), under one rocprofv3 --pmc pass per counter set, and prints bytes per launch under each reading next
to the known / algorithmic bytes.

    python tools/traffic_calib.py [--out gpurun_out/traffic]     (the GPU box; spawns rocprofv3)
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ROWS = 8 << 20            # 8 Mi rows of 128 B = 1 GiB, 4x the 256 MiB Infinity Cache
LAUNCHES = 6
PASSES = (
    ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"],
    ["TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_EA0_RDREQ_GMI_32B_sum", "TCC_EA0_RDREQ_IO_32B_sum", "TCC_BUBBLE_sum"],
    ["FETCH_SIZE"],
    ["WRITE_SIZE", "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"],
)
KERNELS = r"calib_stream|calib_halfline|calib_fullline|lds_rollout_kernel|lds_replay_kernel"


def probe():
    import numpy as np  # noqa: F401
    import torch
    import bench
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "calib", "libcalib.so"))
    lib.calib_run.restype = ctypes.c_int
    lib.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                              ctypes.c_void_p]
    tab = torch.zeros(ROWS * 32, dtype=torch.float32, device=dev)
    out = torch.zeros(1 << 20, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for which in (0, 1, 2):
        for _ in range(LAUNCHES):
            assert lib.calib_run(which, tab.data_ptr(), ROWS, 8, out.data_ptr(), s) == 0
    torch.cuda.synchronize()
    del tab
    for cfg in (2, 6):
        a = argparse.Namespace(config=cfg, envs=bench.CONFIGS[cfg]["envs"], seed=42)
        env = bench.make_env(a, dev)
        acts = bench.bench_actions(a.envs, 0, dev)
        for _ in range(LAUNCHES):
            env.rollout(acts)
        torch.cuda.synchronize()
        env.close()


def collect(counters):
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", td, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--probe"]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=300,
                       cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
        rows = {}
        for fn in glob.glob(os.path.join(td, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as fh:
                for r in csv.DictReader(fh):
                    m = re.search(KERNELS, r.get("Kernel_Name", ""))
                    if m and r.get("Counter_Name") in counters:
                        rows.setdefault(m.group(0), {}).setdefault(r["Counter_Name"], []).append(
                            float(r["Counter_Value"]))
    # the first 2 dispatches of each kernel are warm-up
    return {k: {c: sum(v[2:]) / len(v[2:]) for c, v in d.items() if len(v) > 2} for k, d in rows.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "traffic"))
    args = ap.parse_args()
    if args.probe:
        probe()
        return
    import bench
    res = {}
    for counters in PASSES:
        for k, d in collect(counters).items():
            res.setdefault(k, {}).update(d)
    gib = float(ROWS * 128)
    known = {"calib_stream": gib, "calib_halfline": gib, "calib_fullline": gib}
    for cfg, kn in ((2, "lds_rollout_kernel"), (6, "lds_replay_kernel")):
        c = bench.CONFIGS[cfg]
        rf = bench.roofline("rollout", c["envs"], 1.0, 256, market=c["mode"], lds=True)
        known[kn] = float(rf["kernel_bytes_per_launch"])   # reads + writes: the ratio is printed on the total
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out + ".json", "w") as fh:
        json.dump(dict(raw=res, known_bytes=known), fh, indent=1)
    print("per launch, MB (1e6 B); known = the calibration kernels' read bytes / the env kernels' "
          "algorithmic read + write bytes")
    print(f"{'kernel':20s} {'known':>9s} {'FETCH':>9s} {'2xFETCH':>9s} {'sized rd':>9s} {'DRAM32 rd':>9s} "
          f"{'GMI32':>7s} {'IO32':>7s} {'WRITE':>8s} {'req 32/64/128 B (M)':>22s}")
    for k, d in sorted(res.items()):
        g = lambda n: d.get(n, float("nan"))  # noqa: E731
        sized = 32 * g("TCC_EA0_RDREQ_32B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 128 * g("TCC_EA0_RDREQ_128B_sum")
        fetch = g("FETCH_SIZE") * 1024
        wr = g("WRITE_SIZE") * 1024
        print(f"{k:20s} {known.get(k, float('nan')) / 1e6:9.1f} {fetch / 1e6:9.1f} {2 * fetch / 1e6:9.1f} "
              f"{sized / 1e6:9.1f} {32 * g('TCC_EA0_RDREQ_DRAM_32B_sum') / 1e6:9.1f} "
              f"{32 * g('TCC_EA0_RDREQ_GMI_32B_sum') / 1e6:7.1f} {32 * g('TCC_EA0_RDREQ_IO_32B_sum') / 1e6:7.1f} "
              f"{wr / 1e6:8.1f} {g('TCC_EA0_RDREQ_32B_sum') / 1e6:6.2f}/{g('TCC_EA0_RDREQ_64B_sum') / 1e6:6.2f}/"
              f"{g('TCC_EA0_RDREQ_128B_sum') / 1e6:6.2f}")
        if k in ("lds_rollout_kernel", "lds_replay_kernel"):
            kb = known[k]
            print(f"{'':20s} traffic / algorithmic: 2xFETCH+WRITE {(2 * fetch + wr) / kb:.3f}, "
                  f"sized reads+WRITE {(sized + wr) / kb:.3f}, DRAM32 reads+WRITE "
                  f"{(32 * g('TCC_EA0_RDREQ_DRAM_32B_sum') + wr) / kb:.3f}")


if __name__ == "__main__":
    main()
