#!/bin/bash
# LDS-rollout iteration: the rollout / LDS parity tests, then the A/B of tools/ab/*.so
set -o pipefail
TAG=${1:-lds}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lds or rollout or state or fused or full_size or sharding or odd or summar or closed_loop" > $O/pytest.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab.sh $TAG
