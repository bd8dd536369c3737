#!/usr/bin/env python3
"""Per-kernel busy time and overlap from a rocprofv3 --kernel-trace CSV directory:
for every kernel name the mean duration, and the union-of-intervals wall time of the
last dispatches vs the sum of their durations (how much of them ran concurrently).
Usage: python tools/timeline.py DIR"""
import csv
import glob
import os
import sys


def short(n):
    for k in ("lds_rollout_kernel", "step_market_kernel", "step1_kernel", "step_kernel", "market_kernel"):
        if k in n:
            return k
    return None


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # the rollout phase: from the first to the last rollout kernel (he_step runs of the
    # bench's secondary measurements, step1_kernel, excluded), second half = steady state
    roll = [r for r in rows if r[2] in ("step_kernel", "step_market_kernel", "lds_rollout_kernel")]
    if roll:
        lo, hi = roll[len(roll) // 2][0], roll[-1][1]
        rows = [r for r in rows if r[2] != "step1_kernel" and r[0] >= lo and r[1] <= hi]
    else:
        rows = rows[len(rows) // 2:]
    by = {}
    for s, e, k in rows:
        by.setdefault(k, []).append(e - s)
    for k, v in by.items():
        print(f"  {k:20s} n={len(v):4d} mean {sum(v) / len(v) / 1e3:9.1f} us")
    tot = sum(e - s for s, e, _ in rows)
    union, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    print(f"  sum of durations {tot / 1e6:.3f} ms, busy (union) {union / 1e6:.3f} ms, span {span / 1e6:.3f} ms, "
          f"overlap {1 - union / tot:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
