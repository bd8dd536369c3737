#!/bin/bash
# Round 5: obs-stepper A/B (tools/ab/obs{1,2,3}.so: f32 quotients / reset-row branch / both), then
# the GPU suite on the combined variant
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-obs}; mkdir -p $O; export TMPDIR=/tmp
REPS=${REPS:-3} bash tools/gpu/r05_ab3.sh ${1:-obs} "" "2" obs1 obs2 obs3 || exit 1
CANTORRL_HEDGEENV_LIB=$R/tools/ab/obs3.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_obs3.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest_obs3.log | head -20; tail -20 $O/pytest_obs3.log; exit 1; }
tail -1 $O/pytest_obs3.log
