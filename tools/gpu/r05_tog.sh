#!/bin/bash
# Round 5: book producers' priority pattern -- role timing of the default and the tog build on
# configs 4 and 5, then same-box A/B (tools/ab/tog.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-tog}; mkdir -p $O; export TMPDIR=/tmp
declare -A NE=([4]=524288 [5]=131072)
for c in 4 5; do
  for v in timing timing_tog; do
    CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_timing.py ${NE[$c]} 256 $c > $O/roles_${v}_cfg$c.log 2>&1 || { tail -5 $O/roles_${v}_cfg$c.log; exit 1; }
    echo "$v config $c"; grep -E "^prod|^reward|^obs" $O/roles_${v}_cfg$c.log
  done
done
REPS=${REPS:-2} bash tools/gpu/r05_ab3.sh ${1:-tog} "" "4 5" tog
