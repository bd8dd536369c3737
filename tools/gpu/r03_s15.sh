#!/bin/bash
# Round 3 step 15: Params fields pinned in SGPRs for the generic steppers and the Heston / book
# producers (pin.so, HE_LDS_PIN) -- LDS parity of that build, then configs 5 and 4 A/B.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s15.sh <tag>
set -o pipefail
TAG=${1:-s15}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pin build parity"
CANTORRL_HEDGEENV_LIB=$R/tools/ab/pin.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds_rollout_equals or full_size_slice or heston or book or closed_loop or fixed_european" --timeout 200 --timeout-method thread > $O/pytest_pin.log 2>&1 \
  || { echo "pin parity failed"; grep -E "FAIL|Error|assert" $O/pytest_pin.log | head -30; tail -40 $O/pytest_pin.log; exit 1; }
tail -1 $O/pytest_pin.log
bash tools/gpu/ab_head.sh $TAG 5 pin || exit 1
bash tools/gpu/ab_head.sh $TAG 4 pin || exit 1
echo "[$(date +%T)] done"
