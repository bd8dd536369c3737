#!/bin/bash
# rollout with the market kernel in-stream (no overlap): each kernel's standalone time
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for l in tools/ab/*.so; do b=$(basename $l .so)
  STEP_BENCH_NOPF=1 STEP_BENCH_ROLLOUT=64 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof/${b}_nopf -o run --output-format csv -- ./tools/step_bench 65536 $l > gpurun_out/abprof_${b}_nopf.log 2>&1 || { cat gpurun_out/abprof_${b}_nopf.log; exit 1; }
  grep us/step gpurun_out/abprof_${b}_nopf.log
  python3 tools/kstats.py gpurun_out/abprof/${b}_nopf | head -3
done
