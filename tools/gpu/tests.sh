#!/bin/bash
# GPU parity suite only
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-tests}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
grep -E "fused_rollouts|passed|failed" $O/pytest_gpu.log | tail -4
