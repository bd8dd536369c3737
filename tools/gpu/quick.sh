#!/bin/bash
# GPU parity suite, then the headline bench (no PMC / CPU legs) on the default path and
# with HE_LDS_ROLLOUT=0 (the market-tile kernels) for an A/B on the same box.
#   gpurun --timeout 900 -- bash tools/gpu/quick.sh <tag>
set -o pipefail
TAG=${1:-quick}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for c in 2 3; do
  echo "[$(date +%T)] bench config $c"
  timeout -k 10 200 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api > $O/b_cfg$c.log 2>&1 || { tail -20 $O/b_cfg$c.log; exit 1; }
  grep "^{" $O/b_cfg$c.log
  HE_LDS_ROLLOUT=0 timeout -k 10 200 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api > $O/b_cfg${c}_tile.log 2>&1 || { tail -20 $O/b_cfg${c}_tile.log; exit 1; }
  grep "^{" $O/b_cfg${c}_tile.log
done
echo "[$(date +%T)] done"
