#!/bin/bash
# Round 3 step 28: he_step split A/B, kernel durations from rocprof (graph mode) and 3 more
# value reps.   gpurun --timeout 900 -- bash tools/gpu/r03_s28.sh <tag>
set -o pipefail
TAG=${1:-s28}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_single_env.py -m gpu -x -q -k "split_step or gbm_matches or gbm_mse or rollout_equals_repeated or odd_sizes or greeks_site or closed_loop or single_env or partial_reset or fused_rollouts_mixed" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in base nosplit; do
  lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
  CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 -u bench.py --mode graph --steps 2560 --no-pmc --no-cpu-baseline --no-step-api > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); grep -E "step1|Name" $f | cut -c1-200
done
for rep in 1 2 3; do
  for v in base nosplit latebar nopin; do
    lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
    CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --mode graph --steps 2560 --no-pmc --no-cpu-baseline --no-step-api > $O/g_${v}_$rep.log 2>&1 || { tail -5 $O/g_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; print(sys.argv[1], '%.4g'%d['value'], d['ms_per_step'], r['kernel_us'], r.get('kernel_us_timed_region'))
" $O/g_${v}_$rep.log
  done
done
echo "[$(date +%T)] done"
