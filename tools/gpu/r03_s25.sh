#!/bin/bash
# Round 3 step 25: non-volatile opaque pins (schedulable) -- config 2 A/B: base (volatile pins in
# greeks_lean / lag_return), opq_nv (those non-volatile), rowopq_nv (+ the obs row pinned,
# non-volatile), all_nv (both); parity of all_nv.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s25.sh <tag>
set -o pipefail
TAG=${1:-s25}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
CANTORRL_HEDGEENV_LIB=$R/tools/ab/all_nv.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds_rollout_equals or full_size_slice or closed_loop" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_head.sh $TAG 2 opq_nv rowopq_nv all_nv || exit 1
echo "[$(date +%T)] done"
