#!/bin/bash
# Round 3 step 27: he_step split by role (step1_split_kernel) -- parity (split == step1,
# he_step tests against the oracle and golden vectors), then the graph-mode A/B against
# a build without it.   gpurun --timeout 900 -- bash tools/gpu/r03_s27.sh <tag>
set -o pipefail
TAG=${1:-s27}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_single_env.py -m gpu -x -q -k "split_step or gbm_matches or gbm_mse or rollout_equals_repeated or odd_sizes or greeks_site or closed_loop or single_env or partial_reset or fused_rollouts_mixed" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "parity failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/ab_graph.sh $TAG nosplit || exit 1
echo "[$(date +%T)] done"
