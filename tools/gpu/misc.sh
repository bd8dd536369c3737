#!/bin/bash
# VecNormalize tests + timing, then the LDS book kernel's role timing and PMC (config 4).
set -o pipefail
TAG=${1:-misc}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vecnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_vn.log 2>&1 || { tail -30 $O/pytest_vn.log; exit 1; }
tail -1 $O/pytest_vn.log
timeout -k 10 200 python -u tools/aux_time.py > $O/aux_time.log 2>&1 || { tail -20 $O/aux_time.log; exit 1; }
cat $O/aux_time.log
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 200 python tools/lds_timing.py 524288 256 4 || exit 1
timeout -k 10 400 bash tools/gpu/pmc.sh $TAG/pmc4 --config 4 > $O/pmc4.log 2>&1 || { tail -20 $O/pmc4.log; exit 1; }
grep -A40 "lds_rollout_kernel" $O/pmc4.log | head -40
