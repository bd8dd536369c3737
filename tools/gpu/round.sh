#!/bin/bash
# Measurement pass on the GPU box: GPU parity suite, smoke, default bench (PMC traffic +
# CPU baseline, graph-mode step API), and a rocprofv3 kernel-trace summary of the default bench.
#   gpurun --timeout 1100 -- bash tools/gpu/round.sh <tag>
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[$(date +%T)] smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[$(date +%T)] bench default"
timeout -k 10 400 python -u bench.py > $O/b_default.log 2>&1 || { tail -20 $O/b_default.log; exit 1; }
grep "^{" $O/b_default.log
echo "[$(date +%T)] rocprofv3 kernel trace"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pmc --no-step-api > $R/$O/b_prof.log 2>&1 || { tail -20 $R/$O/b_prof.log; exit 1; }
grep "^{" $R/$O/b_prof.log
find $R/$O/prof -name "*kernel_stats.csv"
echo "[$(date +%T)] done"
