#!/bin/bash
# VALU counters of the MC mark kernel (one --pmc pass, kernel trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-rbpmc}; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/$O/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/rb_time.py 128 > $GRAFT_REPO_ROOT/$O/pmc.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/pmc.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/pmc -name "*counter_collection.csv" | head -1); echo $f
python3 - $f <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", "")[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "mc_kernel" in k:
        print(k, {c: "%.4g" % v for c, v in d.items()})
PY
