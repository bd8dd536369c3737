#!/bin/bash
# A/B of libhedgeenv builds under tools/ab/*.so (graph-mode he_step, GBM)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
N=${1:-65536}
libs=$(ls tools/ab/*.so)
timeout -k 10 120 ./tools/step_bench $N $libs $libs > gpurun_out/step_ab.log 2>&1 || { cat gpurun_out/step_ab.log; exit 1; }
STEP_BENCH_PREFETCH=1 timeout -k 10 120 ./tools/step_bench $N $libs >> gpurun_out/step_ab.log 2>&1 || { cat gpurun_out/step_ab.log; exit 1; }
STEP_BENCH_NO_OBS=1 timeout -k 10 120 ./tools/step_bench $N $libs >> gpurun_out/step_ab.log 2>&1 || { cat gpurun_out/step_ab.log; exit 1; }
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  for l in $libs; do b=$(basename $l .so)
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_$b -o run --output-format csv -- ./tools/step_bench $N $l > /dev/null 2>&1 || exit 1
    STEP_BENCH_PREFETCH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_${b}_pf -o run --output-format csv -- ./tools/step_bench $N $l > /dev/null 2>&1 || exit 1
  done
fi
cat gpurun_out/step_ab.log
