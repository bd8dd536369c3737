#!/bin/bash
# Round 3 step 43: the barrier formula's (H/S) powers through exp_book_g (HE_BOOK_EXP_FAST_UO)
# -- book parity on the newuo build, then config 5 A/B (base = exp_k).
#   gpurun --timeout 900 -- bash tools/gpu/r03_s43.sh <tag>
set -o pipefail
TAG=${1:-s43}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
CANTORRL_HEDGEENV_LIB=$R/tools/ab/newuo.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "book or lds_rollout_equals or full_size_slice or random_configs" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_head.sh $TAG 5 newuo || exit 1
echo "[$(date +%T)] done"
