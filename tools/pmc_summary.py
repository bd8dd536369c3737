#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (step_kernel / market_kernel).
Usage: python tools/pmc_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import sys


def kname(n):
    if "step1_kernel" in n:
        return "step_kernel"
    for k in ("lds_rollout_kernel", "step_market_kernel", "step_kernel", "market_kernel", "reset_kernel",
              "table_greeks_kernel", "init_reset_kernel"):
        if k in n:
            return k
    return None


def main(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                if not k:
                    continue
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[k] = dict(vgpr=r["VGPR_Count"], sgpr=r["SGPR_Count"], lds=r["LDS_Block_Size"],
                               grid=r["Grid_Size"], wg=r["Workgroup_Size"])
    for k, d in agg.items():
        a = {c: sum(v) / len(v) for c, v in d.items()}
        print(f"== {k} {meta[k]} dispatches~{max(len(v) for v in d.values())}")
        W = a.get("SQ_WAVES")
        for c in sorted(a):
            extra = f"   per-wave {a[c] / W:10.1f}" if W and c != "SQ_WAVES" else ""
            print(f"   {c:26s} {a[c]:16.1f}{extra}")


if __name__ == "__main__":
    main(sys.argv[1:])
