#!/bin/bash
# Round 3 step 14: replay FAST steppers on constants pinned in VGPRs -- parity, config 6 A/B
# against the previous build (rprev), role timing of config 6.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s14.sh <tag>
set -o pipefail
TAG=${1:-s14}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] replay parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lds_replay or replay_slice or replay_matches" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
bash tools/gpu/ab_head.sh $TAG 6 rprev || exit 1
echo "[$(date +%T)] role timing config 6"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 6 > $O/role_timing6.log 2>&1 || { tail -5 $O/role_timing6.log; exit 1; }
grep -v amdgpu.ids $O/role_timing6.log
echo "[$(date +%T)] done"
