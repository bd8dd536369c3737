#!/bin/bash
# Round 3 step 11: FAST replay steppers -- parity, config 6 A/B (rslow: generic steppers; rp3:
# reward priority 3; rdiag1: no table reads), role timing of config 6, he_step wave timing.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s11.sh <tag>
set -o pipefail
TAG=${1:-s11}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] replay LDS parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lds_replay or replay_slice or replay_matches" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
bash tools/gpu/ab_head.sh $TAG 6 rslow rp3 rdiag1 || exit 1
echo "[$(date +%T)] role timing config 6"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 6 > $O/role_timing6.log 2>&1 || { tail -5 $O/role_timing6.log; exit 1; }
grep -v amdgpu.ids $O/role_timing6.log
echo "[$(date +%T)] he_step wave timing"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/steptim.so timeout -k 10 120 python tools/step_timing.py 65536 > $O/step_timing.log 2>&1 || { tail -5 $O/step_timing.log; exit 1; }
grep -v amdgpu.ids $O/step_timing.log
echo "[$(date +%T)] done"
