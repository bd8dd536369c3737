#!/bin/bash
# Configs 4/5 (liability book): kernel timeline (rocprofv3 --kernel-trace) of the bench and
# the PMC instruction mix of market_kernel / step_kernel.
#   gpurun --timeout 900 -- bash tools/gpu/book.sh <tag> [configs]
set -o pipefail
TAG=${1:-book}; CFGS=${2:-4 5}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for c in $CFGS; do
  echo "[$(date +%T)] config $c timeline"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tl$c -o run -- python3 $R/bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api --steps 512 --warmup 128 > $O/tl$c.log 2>&1 || { tail -20 $O/tl$c.log; exit 1; }
  cd $R
  grep "^{" $O/tl$c.log
  python3 tools/timeline.py $O/tl$c
  echo "[$(date +%T)] config $c pmc"
  timeout -k 10 400 bash tools/gpu/pmc.sh $TAG/pmc$c --config $c > $O/pmc$c.log 2>&1 || { tail -20 $O/pmc$c.log; exit 1; }
  cat $O/pmc$c.log
done
