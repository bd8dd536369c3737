#!/bin/bash
# Round 3 step 18: replay rows' obs greeks through greeks_fast (table_greeks_kernel and the LDS
# loaders) -- the replay goldens and every GPU test, config 6 A/B against the f64-greeks build
# (rprev) and reward priorities 2 / 3, role timing at priority 0 and 3.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s18.sh <tag>
set -o pipefail
TAG=${1:-s18}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] replay parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lds_replay or replay_slice or replay_matches or policy_rollout_matches" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
echo "[$(date +%T)] suite"
bash tools/gpu/tests.sh $TAG || exit 1
bash tools/gpu/ab_head.sh $TAG 6 rprev rp2 rp3 || exit 1
for t in timing timing_rp3; do
  echo "[$(date +%T)] role timing config 6 $t"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$t.so timeout -k 10 120 python tools/lds_timing.py 65536 256 6 > $O/role6_$t.log 2>&1 || { tail -5 $O/role6_$t.log; exit 1; }
  grep -v amdgpu.ids $O/role6_$t.log
done
echo "[$(date +%T)] done"
