#!/bin/bash
# Round 3 step 40: the book's phi through exp_book and N(d) by copysign (HE_BOOK_EXP_FAST,
# HE_BOOK_NCDF_FAST) -- book parity on the default build, then configs 4 and 5 against each off.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s40.sh <tag>
set -o pipefail
TAG=${1:-s40}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "book or lds_rollout_equals or full_size_slice or random_configs" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_head.sh $TAG 4 oldexp || exit 1
bash tools/gpu/ab_head.sh $TAG 5 oldexp || exit 1
echo "[$(date +%T)] done"
