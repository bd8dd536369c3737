#!/bin/bash
# Round measurement: GPU parity suite, smoke, default bench (PMC + CPU baseline), rocprofv3
# kernel-trace summary of the default bench, configs 3/4/5
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/b_default.log 2>&1 || { tail -20 $O/b_default.log; exit 1; }
grep "^{" $O/b_default.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pmc --no-step-api > $R/$O/b_prof.log 2>&1 || { tail -20 $R/$O/b_prof.log; exit 1; }
grep "^{" $R/$O/b_prof.log
cd $R
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-step-api > $O/b_cfg$c.log 2>&1 || { tail -20 $O/b_cfg$c.log; exit 1; }
  grep "^{" $O/b_cfg$c.log
done
