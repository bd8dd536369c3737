#!/bin/bash
# Round 5: same-box A/B of tools/ab/<variant>.so against the default library on the given
# configs, then the GPU suite on the variant
#   gpurun -- bash tools/gpu/r05_var.sh <tag> <variant> "<configs>"
set -o pipefail
TAG=${1:-var}; V=$2; CFGS=${3:-"2"}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
REPS=${REPS:-3} bash tools/gpu/r05_ab3.sh $TAG "" "$CFGS" $V || exit 1
CANTORRL_HEDGEENV_LIB=$R/tools/ab/$V.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_$V.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest_$V.log | head -20; tail -20 $O/pytest_$V.log; exit 1; }
tail -1 $O/pytest_$V.log
