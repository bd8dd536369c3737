#!/bin/bash
# Round 3 step 20: alternating producer priorities (alt), with the lagged obs stepper (lagalt):
# parity of lagalt, config 2 A/B (base, alt, lag, lagalt), role timing of alt / lagalt.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s20.sh <tag>
set -o pipefail
TAG=${1:-s20}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] lagalt parity"
CANTORRL_HEDGEENV_LIB=$R/tools/ab/lagalt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds_rollout_equals or full_size_slice or closed_loop" --timeout 200 --timeout-method thread > $O/pytest_lagalt.log 2>&1 \
  || { echo "lagalt parity failed"; grep -E "FAIL|Error|assert" $O/pytest_lagalt.log | head -30; tail -40 $O/pytest_lagalt.log; exit 1; }
tail -1 $O/pytest_lagalt.log
bash tools/gpu/ab_head.sh $TAG 2 alt lag lagalt || exit 1
for t in timing_alt timing_lagalt; do
  echo "[$(date +%T)] role timing config 2 $t"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$t.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role2_$t.log 2>&1 || { tail -5 $O/role2_$t.log; exit 1; }
  grep -v amdgpu.ids $O/role2_$t.log
done
echo "[$(date +%T)] done"
# replay: the new-episode rows loaded only by the lanes whose episode ends in the block
echo "[$(date +%T)] replay parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds_replay or replay_slice" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
bash tools/gpu/ab_head.sh $TAG 6 rprev || exit 1
timeout -k 10 400 python -u bench.py --config 6 --no-cpu-baseline --no-step-api > $O/b6_pmc.log 2>&1 || { tail -20 $O/b6_pmc.log; exit 1; }
grep -o '"traffic_over_bytes": [0-9.]*' $O/b6_pmc.log
echo "[$(date +%T)] done replay"
