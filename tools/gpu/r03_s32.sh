#!/bin/bash
# Round 3 step 32: vn_apply_kernel with R rows per thread (1 / R of the workgroups merge the
# partials) -- VecNormalize parity on R = 4, then rocprof kernel stats of tools/aux_time.py
# for R = 1 (base), 2, 4.    gpurun --timeout 900 -- bash tools/gpu/r03_s32.sh <tag>
set -o pipefail
TAG=${1:-s32}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for v in vnr4 vnr2; do
  CANTORRL_HEDGEENV_LIB=$R/tools/ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_vecnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 \
    || { echo "vecnorm parity failed ($v)"; tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for rep in 1 2; do
for v in base vnr2 vnr4; do
  lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
  CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$rep -o run -- python3 -u tools/aux_time.py > $O/aux_${v}_$rep.log 2>&1 || { tail -5 $O/aux_${v}_$rep.log; exit 1; }
  f=$(find $O/prof_${v}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'vn_' in r['Name'] or 'step1' in r['Name']: print(sys.argv[2], r['Name'][:48], r['Calls'], r['AverageNs'], r['MinNs'])
" $f $v
  grep -E "apply|vecnorm_step|fused" $O/aux_${v}_$rep.log
done
done
echo "[$(date +%T)] done"
