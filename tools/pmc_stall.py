#!/usr/bin/env python3
"""Where the waves of the dominant kernel spend their cycles: one rocprofv3 --pmc pass per
counter group over `bench.py --probe` (SQ wave-state counters count quad-cycles,
MI355X_MICROARCH.md), printed per kernel as fractions of SQ_WAVE_CYCLES.

    python tools/pmc_stall.py [--config C] [--envs N]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

GROUPS = [
    ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"],
    ["SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD",
     "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_SCA"],
    ["SQ_WAVE_CYCLES", "SQC_ICACHE_REQ", "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE",
     "SQ_IFETCH", "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_SALU"],
]
if os.environ.get("PMC_GROUPS"):  # e.g. PMC_GROUPS=2 for the instruction-cache group only
    GROUPS = [GROUPS[int(k)] for k in os.environ["PMC_GROUPS"].split(",")]

args = bench.parse(sys.argv[1:])
cfg = bench.CONFIGS[args.config]
args.envs = args.envs or cfg["envs"]
if args.rollout_k is None:
    args.rollout_k = 256 if bench.lds_rollout(cfg) else bench.M_BLOCK
out = {}
for g in GROUPS:
    res, err = bench.pmc_pass(args, g, bench.STEP_KERNELS)
    if res is None:
        print("pass failed:", err, flush=True)
        continue
    for k, d in res.items():
        out.setdefault(k, {}).update(d)
for k, d in out.items():
    wc = d.get("SQ_WAVE_CYCLES") or 1.0
    print(k, json.dumps({c: (round(v / wc, 4) if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else v)
                         for c, v in d.items()}), flush=True)
