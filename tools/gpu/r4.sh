#!/bin/bash
# Round-1 measurement pass: GPU parity suite, default bench (PMC + CPU baseline),
# configs 3/5, rollout mode, and a rocprofv3 kernel-trace summary of the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/b_default.log 2>&1 || exit 1
grep "^{" gpurun_out/b_default.log
timeout -k 10 300 python bench.py --config 3 --steps 640 --warmup 128 --no-cpu-baseline > gpurun_out/b_cfg3.log 2>&1 || exit 1
grep "^{" gpurun_out/b_cfg3.log
timeout -k 10 300 python bench.py --config 5 --steps 640 --warmup 128 --no-cpu-baseline > gpurun_out/b_cfg5.log 2>&1 || exit 1
grep "^{" gpurun_out/b_cfg5.log
timeout -k 10 300 python bench.py --mode rollout --no-cpu-baseline --no-pmc > gpurun_out/b_rollout.log 2>&1 || exit 1
grep "^{" gpurun_out/b_rollout.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > gpurun_out/b_prof.log 2>&1 || exit 1
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
