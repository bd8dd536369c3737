#!/bin/bash
# Round 5: tail diagnostics (tools/abt/<tail variants>.so, tools/lds_tail.py), then same-box A/B of
# tools/ab/<variants>.so against this tree on the given configs (alternating, two repetitions).
#   gpurun --timeout 1200 -- bash tools/gpu/r05_ab2.sh <tag> "<tail variants>" "<configs>" <variant>...
set -o pipefail
TAG=${1:-ab2}; TV=${2:-""}; CFGS=${3:-"2"}; shift 3
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for v in $TV; do
  echo "[$(date +%T)] tail $v"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_tail.py --out $O/$v > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  grep -v amdgpu.ids $O/$v.log | head -4
done
for c in $CFGS; do
  for rep in 1 2; do
    for v in base "$@"; do
      lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
      CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api --no-sb3-api > $O/b${c}_${v}_$rep.log 2>&1 || { tail -5 $O/b${c}_${v}_$rep.log; exit 1; }
      python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1].split('/')[-1], '%.4g'%d['value'], d['roofline']['kernel_us'], (d.get('shard_check') or {}).get('result'))
" $O/b${c}_${v}_$rep.log
    done
  done
done
echo "[$(date +%T)] done"
