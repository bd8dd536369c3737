#!/bin/bash
# Round 5: role timing + workgroup spread (tools/abt/<timing variants>.so, tools/lds_timing.py) on
# config 2, then same-box A/B of tools/ab/<variants>.so on the given configs (alternating, REPS).
#   gpurun --timeout 1200 -- bash tools/gpu/r05_ab3.sh <tag> "<timing variants>" "<configs>" <variant>...
set -o pipefail
TAG=${1:-ab3}; TV=${2:-""}; CFGS=${3:-"2"}; shift 3
REPS=${REPS:-2}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for v in $TV; do
  echo "[$(date +%T)] role timing $v"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_timing.py 65536 256 2 > $O/roles_$v.log 2>&1 || { tail -5 $O/roles_$v.log; exit 1; }
  grep -v amdgpu.ids $O/roles_$v.log
done
for c in $CFGS; do
  for rep in $(seq 1 $REPS); do
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
