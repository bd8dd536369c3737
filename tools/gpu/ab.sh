#!/bin/bash
# A/B of builds: the headline bench (kernel time of the dominant kernel) with the in-tree
# library and with every tools/ab/*.so (CANTORRL_HEDGEENV_LIB), configs $CFGS (default 2 3).
#   gpurun --timeout 900 -- bash tools/gpu/ab.sh <tag>
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for c in ${CFGS:-2 3 4}; do
  for l in default tools/ab/*.so; do
    b=$(basename $l .so)
    if [ "$l" = default ]; then unset CANTORRL_HEDGEENV_LIB; else export CANTORRL_HEDGEENV_LIB=$R/$l; fi
    timeout -k 10 200 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api $BENCH_ARGS > $O/b_${b}_cfg$c.log 2>&1 || { tail -20 $O/b_${b}_cfg$c.log; exit 1; }
    python3 -c "
import json,sys
l=[json.loads(x) for x in open('$O/b_${b}_cfg$c.log') if x.startswith('{')][0]
r=l['roofline']
print('cfg $c %-14s value %.4g  kernel_us %9.2f  frac %.4f  K %s' % ('$b', l['value'], r['kernel_us'], r['frac'], l['config']['rollout_k']))
"
  done
done
