#!/bin/bash
# VecNormalize tests + timing; LDS role timing and PMC mix of the headline config.
set -o pipefail
TAG=${1:-diag2}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vecnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_vn.log 2>&1 || { tail -30 $O/pytest_vn.log; exit 1; }
tail -1 $O/pytest_vn.log
timeout -k 10 200 python -u tools/aux_time.py > $O/aux_time.log 2>&1 || { tail -20 $O/aux_time.log; exit 1; }
head -3 $O/aux_time.log
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 200 python tools/lds_timing.py 65536 256 2 || exit 1
timeout -k 10 400 bash tools/gpu/pmc.sh $TAG/pmc2 --config 2 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
grep -A40 "lds_rollout_kernel" $O/pmc2.log | head -40
