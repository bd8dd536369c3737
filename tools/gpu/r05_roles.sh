#!/bin/bash
# Role timing (-DHE_LDS_TIMING builds under tools/abt/<variant>.so) of lds_rollout_kernel per
# bench config, then same-box A/B of tools/ab/<variant>.so against this tree's library:
#   gpurun -- bash tools/gpu/r05_roles.sh <tag> "<timing variants>" "<configs>" <ab variant>...
set -o pipefail
TAG=${1:-roles}; TV=${2:-timing}; CFGS=${3:-"2 4 5"}; shift 3
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
declare -A NE=([2]=65536 [3]=1048576 [4]=524288 [5]=131072 [6]=65536)
for c in $CFGS; do
  for v in $TV; do
    echo "[$(date +%T)] role timing $v config $c"
    CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_timing.py ${NE[$c]} 256 $c > $O/roles_${v}_cfg$c.log 2>&1 || { tail -5 $O/roles_${v}_cfg$c.log; exit 1; }
    grep -v amdgpu.ids $O/roles_${v}_cfg$c.log
  done
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
