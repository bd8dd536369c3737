#!/bin/bash
# Round 3 step 23: wave-uniform fast-path checks in the lockstep math (ndtr_pair_n, log_ratio_n,
# exp_k_n) -- LDS parity, config 2 and 4 A/B against the lane-wise checks, role timing.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s23.sh <tag>
set -o pipefail
TAG=${1:-s23}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rng.py -m gpu -x -q -k "lds or full_size or closed_loop or gbm_matches or device" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_head.sh $TAG 2 lanewise || exit 1
bash tools/gpu/ab_head.sh $TAG 4 lanewise || exit 1
echo "[$(date +%T)] role timing config 2"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role2.log 2>&1 || { tail -5 $O/role2.log; exit 1; }
grep -v amdgpu.ids $O/role2.log
echo "[$(date +%T)] done"
