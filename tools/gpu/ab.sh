#!/bin/bash
# A/B of libhedgeenv builds under tools/ab/*.so: graph-mode he_step and he_rollout(K=64),
# GBM, 65,536 envs (or $1).  Then the GPU parity suite on the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
N=${1:-65536}
libs=$(ls tools/ab/*.so)
L=gpurun_out/ab.log
echo "== he_step graph" > $L
timeout -k 10 120 ./tools/step_bench $N $libs >> $L 2>&1 || { cat $L; exit 1; }
echo "== he_rollout K=64" >> $L
STEP_BENCH_ROLLOUT=64 timeout -k 10 120 ./tools/step_bench $N $libs $libs >> $L 2>&1 || { cat $L; exit 1; }
cat $L
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
