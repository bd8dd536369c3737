#!/bin/bash
# Round 3 step 37: the book Mills polynomial at degree 16 (HE_MILLS_DEG16) -- book parity, configs 4 and 5 A/B.
# loop unrolled by 2 -- book parity on the Estrin build, then configs 4 and 5 A/B.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s36.sh <tag>
set -o pipefail
TAG=${1:-s36}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
CANTORRL_HEDGEENV_LIB=$R/tools/ab/deg16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "book or lds_rollout_equals or full_size_slice or random_configs" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_head.sh $TAG 4 deg16 || exit 1
bash tools/gpu/ab_head.sh $TAG 5 deg16 || exit 1
echo "[$(date +%T)] done"
