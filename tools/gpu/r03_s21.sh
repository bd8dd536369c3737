#!/bin/bash
# Round 3 step 21: obs rows stored write-through (sc1 buffer stores, obssc1.so) -- parity, then
# configs 6 and 2 A/B and the PMC traffic of config 6 with it.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s21.sh <tag>
set -o pipefail
TAG=${1:-s21}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
CANTORRL_HEDGEENV_LIB=$R/tools/ab/obssc1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lds_replay or lds_rollout_equals" --timeout 200 --timeout-method thread > $O/pytest_sc1.log 2>&1 \
  || { echo "sc1 parity failed"; grep -E "FAIL|Error|assert" $O/pytest_sc1.log | head -30; tail -40 $O/pytest_sc1.log; exit 1; }
tail -1 $O/pytest_sc1.log
bash tools/gpu/ab_head.sh $TAG 6 obssc1 || exit 1
bash tools/gpu/ab_head.sh $TAG 2 obssc1 || exit 1
CANTORRL_HEDGEENV_LIB=$R/tools/ab/obssc1.so timeout -k 10 400 python -u bench.py --config 6 --no-cpu-baseline --no-step-api > $O/b6_sc1_pmc.log 2>&1 || { tail -20 $O/b6_sc1_pmc.log; exit 1; }
grep -o '"traffic_over_bytes": [0-9.]*' $O/b6_sc1_pmc.log
echo "[$(date +%T)] done"
