#!/bin/bash
# A/B of tools/ab/*.so (he_rollout K=64 and graph he_step, GBM) at 65,536 and 1,048,576 envs
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
hipcc -O2 -o /tmp/step_bench tools/step_bench.cpp -ldl 2>/dev/null || exit 1
libs=$(ls tools/ab/*.so)
L=gpurun_out/ab2.log; : > $L
for N in 65536 1048576; do
  echo "== N=$N he_rollout K=64" >> $L
  STEP_BENCH_ROLLOUT=64 timeout -k 10 120 /tmp/step_bench $N $libs $libs >> $L 2>&1 || { cat $L; exit 1; }
done
echo "== N=65536 he_step graph" >> $L
timeout -k 10 120 /tmp/step_bench 65536 $libs >> $L 2>&1 || { cat $L; exit 1; }
cat $L
