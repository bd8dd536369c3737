#!/bin/bash
# Round 3 step 8 (restored tree): GPU suite, role timing at the default and at reward
# priority 3, same-box A/B of the reward-stepper priority (pC 1, pD 2, pE 3, pH rew 2 + obs 3)
# on configs 2 and 4.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s8.sh <tag>
set -o pipefail
TAG=${1:-s8}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] suite"
bash tools/gpu/tests.sh $TAG || exit 1
for t in timing timing_pE; do
  echo "[$(date +%T)] role timing $t"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$t.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role_$t.log 2>&1 || { tail -5 $O/role_$t.log; exit 1; }
  grep -v amdgpu.ids $O/role_$t.log
done
bash tools/gpu/ab_head.sh $TAG 2 pC pD pE pH || exit 1
bash tools/gpu/ab_head.sh $TAG 4 pC pE || exit 1
echo "[$(date +%T)] done"
