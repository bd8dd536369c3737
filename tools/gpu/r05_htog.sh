#!/bin/bash
# Round 5: Heston book producers' priority pattern -- role timing (tools/abt/timing{,_h4,_h31}.so)
# and same-box A/B (tools/ab/h4.so, h31.so) on config 5
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-htog}; mkdir -p $O; export TMPDIR=/tmp
for v in timing timing_h4 timing_h31; do
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_timing.py 131072 256 5 > $O/roles_${v}_cfg5.log 2>&1 || { tail -5 $O/roles_${v}_cfg5.log; exit 1; }
  echo "$v config 5"; grep -E "^prod|^reward|^obs" $O/roles_${v}_cfg5.log
done
REPS=${REPS:-2} bash tools/gpu/r05_ab3.sh ${1:-htog} "" "5" h4 h31
