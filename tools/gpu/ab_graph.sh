#!/bin/bash
# Same-box A/B of library builds on the Gym-API path (bench --mode graph: one he_step
# launch per step, captured in hipGraphs):  gpurun -- bash tools/gpu/ab_graph.sh <tag> <variant>...
set -o pipefail
TAG=${1:-abg}; shift
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
    CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --mode graph --steps 2560 --no-pmc --no-cpu-baseline --no-step-api > $O/g_${v}_$rep.log 2>&1 || { tail -5 $O/g_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1], '%.4g'%d['value'], d['roofline']['kernel_us'], d['roofline']['frac'])
" $O/g_${v}_$rep.log
  done
done
