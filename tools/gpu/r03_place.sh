#!/bin/bash
# Round 3: fixed-European parity tests on the default build, the wave-role placement dump
# (tools/lds_hwid.py over the -DHE_LDS_HWID builds) and the same-box A/B of the balanced
# placement (tools/ab/bal.so) on configs 2, 4 and 5.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_place.sh <tag>
set -o pipefail
TAG=${1:-place}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] parity: fixed-European marks, closed loops, LDS == tile"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "fixed_european or closed_loop or lds_rollout" > $O/pytest_fe.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_fe.log | head -30; tail -30 $O/pytest_fe.log; exit 1; }
tail -1 $O/pytest_fe.log
for v in hwid hwbal; do
  for c in 2 4; do
    echo "[$(date +%T)] placement $v config $c"
    CANTORRL_HEDGEENV_LIB=$R/tools/ab/$v.so timeout -k 10 120 python -u tools/lds_hwid.py --config $c > $O/hwid_${v}_$c.json 2>$O/hwid_${v}_$c.err \
      || { tail -20 $O/hwid_${v}_$c.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in ('wg_per_cu','distinct_simds','max_obs_waves_per_simd','wave0_simd')})" $O/hwid_${v}_$c.json
  done
done
for c in 2 4 5; do
  echo "[$(date +%T)] A/B config $c"
  bash tools/gpu/ab_head.sh $TAG $c bal || exit 1
done
echo "[$(date +%T)] done"
