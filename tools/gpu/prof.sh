#!/bin/bash
# default bench + rocprofv3 kernel-trace summary of the same command, then the A/B of tools/ab/*.so
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/b_default.log 2>&1 || { tail -20 $O/b_default.log; exit 1; }
grep "^{" $O/b_default.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pmc --no-step-api > $R/$O/b_prof.log 2>&1 || { tail -20 $R/$O/b_prof.log; exit 1; }
grep "^{" $R/$O/b_prof.log
cd $R
if ls tools/ab/*.so >/dev/null 2>&1; then bash tools/gpu/ab2.sh; fi
