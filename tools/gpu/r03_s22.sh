#!/bin/bash
# Round 3 step 22: opaque select operands (greeks_lean, lag_return: no exec-mask branches in the
# obs stepper's block) -- LDS parity, config 2 / 6 A/B against HE_OPAQUE_SEL=0, role timing.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s22.sh <tag>
set -o pipefail
TAG=${1:-s22}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds or full_size or closed_loop or gbm_matches or greeks_site or replay_matches" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_head.sh $TAG 2 noopq || exit 1
bash tools/gpu/ab_head.sh $TAG 6 noopq || exit 1
echo "[$(date +%T)] role timing config 2"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role2.log 2>&1 || { tail -5 $O/role2.log; exit 1; }
grep -v amdgpu.ids $O/role2.log
echo "[$(date +%T)] done"
