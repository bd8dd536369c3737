#!/bin/bash
# rocprofv3 kernel stats of graph-mode he_step (and rollout with ROLL=K) per tools/ab/*.so
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
N=${1:-65536}
for l in tools/ab/*.so; do b=$(basename $l .so)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof/$b -o run --output-format csv -- ./tools/step_bench $N $l > gpurun_out/abprof_$b.log 2>&1 || { cat gpurun_out/abprof_$b.log; exit 1; }
  grep us/step gpurun_out/abprof_$b.log
  python3 tools/kstats.py gpurun_out/abprof/$b
  if [ -n "$ROLL" ]; then
    STEP_BENCH_ROLLOUT=$ROLL timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof/${b}_r -o run --output-format csv -- ./tools/step_bench $N $l > gpurun_out/abprof_${b}_r.log 2>&1 || { cat gpurun_out/abprof_${b}_r.log; exit 1; }
    grep us/step gpurun_out/abprof_${b}_r.log
    python3 tools/kstats.py gpurun_out/abprof/${b}_r
  fi
done
