#!/bin/bash
# Round 3 step 5: the GPU suite on the lockstep-producer tree, then same-box A/B:
# nofull (FULL = 0: per-slot producers, 5 waves/SIMD for GBM) and booklock (GBM book slots in
# lockstep) against the in-tree build on configs 2, 3, 4, 5.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s5.sh <tag>
set -o pipefail
TAG=${1:-s5}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu/ab_head.sh $TAG 2 nofull || exit 1
bash tools/gpu/ab_head.sh $TAG 3 nofull || exit 1
bash tools/gpu/ab_head.sh $TAG 4 nofull booklock || exit 1
bash tools/gpu/ab_head.sh $TAG 5 nofull || exit 1
echo "[$(date +%T)] done"
