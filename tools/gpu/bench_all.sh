#!/bin/bash
# default bench line plus configs 3/4/5 (no CPU baseline, no step API) on the GPU box
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/b_default.log 2>&1 || { tail -20 $O/b_default.log; exit 1; }
grep "^{" $O/b_default.log
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-step-api > $O/b_cfg$c.log 2>&1 || { tail -20 $O/b_cfg$c.log; exit 1; }
  grep "^{" $O/b_cfg$c.log
done
