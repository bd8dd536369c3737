#!/bin/bash
# Round 5: the lagged-obs pipeline (tools/ab/lag.so, lagxor.so: -DHE_LDS_OBS_LAG=1 [+ role XOR])
# -- its parity on the LDS-rollout tests, role timing of config 2, then same-box A/B.
#   gpurun --timeout 1200 -- bash tools/gpu/r05_lag.sh <tag> "<variants>" "<timing variants>"
set -o pipefail
TAG=${1:-lag}; VARS=${2:-"lag lagxor"}; TV=${3:-"timing timing_lag timing_lagxor"}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
K="lds_rollout_equals_tile or full_size_slice or closed_loop or gbm_matches or rollout_equals_repeated or sharding or random_configs_paths or episode_summaries_match or fused_rollouts_mixed"
for v in $VARS; do
  echo "[$(date +%T)] parity with $v"
  CANTORRL_HEDGEENV_LIB=$R/tools/ab/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest_$v.log 2>&1 \
    || { echo "pytest failed ($v)"; grep -E "FAIL|Error|assert" $O/pytest_$v.log | head -30; tail -20 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for v in $TV; do
  echo "[$(date +%T)] role timing $v config 2"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_timing.py 65536 256 2 > $O/roles_${v}_cfg2.log 2>&1 || { tail -5 $O/roles_${v}_cfg2.log; exit 1; }
  grep -v amdgpu.ids $O/roles_${v}_cfg2.log
done
for c in 2 3; do
  for rep in 1 2; do
    for v in base $VARS; do
      [ $c = 3 ] && [ $rep = 2 ] && continue
      lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
      CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api --no-sb3-api > $O/b${c}_${v}_$rep.log 2>&1 || { tail -5 $O/b${c}_${v}_$rep.log; exit 1; }
      python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1].split('/')[-1], '%.4g'%d['value'], d['roofline']['kernel_us'], (d.get('shard_check') or {}).get('result'))
" $O/b${c}_${v}_$rep.log
    done
  done
done
echo "[$(date +%T)] done"
