#!/bin/bash
# Same-box A/B of libhedgeenv variants (tools/ab/<name>.so) on one bench config, then
# the PMC wave-state breakdown (tools/pmc_stall.py) of the default build:
#   gpurun -- bash tools/gpu/ab_head.sh <tag> <config> <variant>...
set -o pipefail
TAG=${1:-abh}; C=${2:-2}; shift 2
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
    CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --config $C --no-pmc --no-cpu-baseline --no-step-api > $O/b${C}_${v}_$rep.log 2>&1 || { tail -5 $O/b${C}_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1], '%.4g'%d['value'], d['roofline']['kernel_us'])
" $O/b${C}_${v}_$rep.log
  done
done
if [ -n "$STALL" ]; then
  for c in $STALL; do timeout -k 10 300 python -u tools/pmc_stall.py --config $c > $O/stall_$c.log 2>&1 || { tail -5 $O/stall_$c.log; exit 1; }; cat $O/stall_$c.log; done
fi
