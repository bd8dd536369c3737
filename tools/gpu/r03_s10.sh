#!/bin/bash
# Round 3 step 10: replay LDS kernel with loader-evaluated greeks -- parity, then same-box A/B on
# config 6 (base = HE_REPLAY_LGREEKS 1; rg0 reads recg; rdiag1 no table reads; rdiag2 steppers
# idle; rp3 reward priority 3; HE_LDS_ROLLOUT=0 step_kernel), role timing of config 2 at the
# new reward priority, the book-kernel reward priority A/B on configs 4 and 5.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s10.sh <tag>
set -o pipefail
TAG=${1:-s10}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] replay LDS parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lds_replay or replay_slice or lds_rollout_equals or full_size_slice" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
bash tools/gpu/ab_head.sh $TAG 6 rg0 rdiag1 rdiag2 rp3 || exit 1
HE_LDS_ROLLOUT=0 timeout -k 10 300 python -u bench.py --config 6 --no-pmc --no-cpu-baseline --no-step-api > $O/b6_tile.log 2>&1 || { tail -5 $O/b6_tile.log; exit 1; }
grep -o '"kernel_us": [0-9.]*' $O/b6_tile.log | head -1
echo "[$(date +%T)] role timing"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role_timing.log 2>&1 || { tail -5 $O/role_timing.log; exit 1; }
grep -v amdgpu.ids $O/role_timing.log
bash tools/gpu/ab_head.sh $TAG 4 bookrew3 || exit 1
bash tools/gpu/ab_head.sh $TAG 5 bookrew3 || exit 1
echo "[$(date +%T)] done"
