#!/bin/bash
# Round 3 step 7: wave-priority permutations (the reward stepper is the critical role since
# the lockstep producers): role timing at (rew 3, obs 2, prod 1) and all-equal, same-box
# A/B of pD..pG on config 2 and pB/pD/pE on configs 4 and 5, wave-state PMC of config 2.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s7.sh <tag>
set -o pipefail
TAG=${1:-s7}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for t in timing timing_pE timing_pG; do
  echo "[$(date +%T)] role timing $t"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$t.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role_$t.log 2>&1 || { tail -5 $O/role_$t.log; exit 1; }
  grep -v amdgpu.ids $O/role_$t.log
done
bash tools/gpu/ab_head.sh $TAG 2 pD pE pF pG || exit 1
bash tools/gpu/ab_head.sh $TAG 4 pB pD pE || exit 1
bash tools/gpu/ab_head.sh $TAG 5 pB pD pE || exit 1
PMC_GROUPS=0 timeout -k 10 300 python -u tools/pmc_stall.py --config 2 > $O/stall_2.log 2>&1 || { tail -5 $O/stall_2.log; exit 1; }
cat $O/stall_2.log
echo "[$(date +%T)] done"
