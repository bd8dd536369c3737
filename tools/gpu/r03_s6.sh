#!/bin/bash
# Round 3 step 6: LDS parity of the obs-lockstep variant, role timing, then same-box A/B of
# wave priorities (pA: producers 2; pB: producers 2, obs 1; pC: reward 1) and obslock.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s6.sh <tag>
set -o pipefail
TAG=${1:-s6}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] obslock parity"
CANTORRL_HEDGEENV_LIB=$R/tools/ab/obslock.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds or LDS or closed" --timeout 300 --timeout-method thread > $O/pytest_obslock.log 2>&1 \
  || { echo "obslock parity failed"; tail -30 $O/pytest_obslock.log; exit 1; }
tail -1 $O/pytest_obslock.log
echo "[$(date +%T)] role timing"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role_timing.log 2>&1 || { tail -5 $O/role_timing.log; exit 1; }
cat $O/role_timing.log
bash tools/gpu/ab_head.sh $TAG 2 pA pB pC obslock || exit 1
bash tools/gpu/ab_head.sh $TAG 4 pA pB || exit 1
echo "[$(date +%T)] done"
