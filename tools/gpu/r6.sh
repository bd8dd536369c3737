#!/bin/bash
# GPU parity suite; default bench; the same with the side-stream market (HE_FUSED_MARKET=0); configs 3/4/5
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $O/b_default.log 2>&1 || { tail -20 $O/b_default.log; exit 1; }
grep "^{" $O/b_default.log
HE_FUSED_MARKET=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-step-api > $O/b_sidestream.log 2>&1 || { tail -20 $O/b_sidestream.log; exit 1; }
grep "^{" $O/b_sidestream.log
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-step-api > $O/b_cfg$c.log 2>&1 || { tail -20 $O/b_cfg$c.log; exit 1; }
  grep "^{" $O/b_cfg$c.log
done
