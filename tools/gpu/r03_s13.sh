#!/bin/bash
# Round 3 step 13: branch-free replay reward stepper (IEEE divisions, select-only autoreset) --
# parity (+ the lagged-obs A/B build's LDS parity), config 6 A/B against the previous build
# (rprev), role timing of config 6; VecNormalize timing against the previous apply kernel (oldvn);
# the producer-wave asymmetry on config 2 (pwswap: env halves swapped; prod1p2: the second
# producer at priority 2; lagp1: lagged obs + prod1p2).
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s13.sh <tag>
set -o pipefail
TAG=${1:-s13}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] replay parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lds_replay or replay_slice or replay_matches" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
echo "[$(date +%T)] lag build parity"
CANTORRL_HEDGEENV_LIB=$R/tools/ab/lag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds_rollout_equals or full_size_slice or closed_loop" --timeout 200 --timeout-method thread > $O/pytest_lag.log 2>&1 \
  || { echo "lag parity failed"; grep -E "FAIL|Error|assert" $O/pytest_lag.log | head -30; tail -40 $O/pytest_lag.log; exit 1; }
tail -1 $O/pytest_lag.log
bash tools/gpu/ab_head.sh $TAG 6 rprev || exit 1
echo "[$(date +%T)] role timing config 6"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 6 > $O/role_timing6.log 2>&1 || { tail -5 $O/role_timing6.log; exit 1; }
grep -v amdgpu.ids $O/role_timing6.log
echo "[$(date +%T)] vecnorm"
timeout -k 10 300 python -u -m pytest tests/test_vecnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_vn.log 2>&1 || { tail -30 $O/pytest_vn.log; exit 1; }
tail -1 $O/pytest_vn.log
for rep in 1 2; do
  for v in base oldvn; do
    lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
    CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 200 python -u tools/aux_time.py > $O/aux_${v}_$rep.log 2>&1 || { tail -20 $O/aux_${v}_$rep.log; exit 1; }
    echo "$v $rep"; grep -E "us/step" $O/aux_${v}_$rep.log
  done
done
bash tools/gpu/ab_head.sh $TAG 2 pwswap prod1p2 lagp1 || exit 1
for t in timing timing_pwswap timing_lagp1; do
  echo "[$(date +%T)] role timing config 2 $t"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$t.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role2_$t.log 2>&1 || { tail -5 $O/role2_$t.log; exit 1; }
  grep -v amdgpu.ids $O/role2_$t.log
done
echo "[$(date +%T)] kernarg preload build: parity + Gym-API A/B"
CANTORRL_HEDGEENV_LIB=$R/tools/ab/kpre.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_single_env.py -m gpu -x -q -k "replay_matches or gbm_matches or single_env or closed_loop" --timeout 200 --timeout-method thread > $O/pytest_kpre.log 2>&1 \
  || { echo "kpre parity failed"; grep -E "FAIL|Error|assert" $O/pytest_kpre.log | head -30; tail -40 $O/pytest_kpre.log; exit 1; }
tail -1 $O/pytest_kpre.log
bash tools/gpu/ab_graph.sh $TAG kpre || exit 1
echo "[$(date +%T)] done"
