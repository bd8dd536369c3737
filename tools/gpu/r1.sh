#!/bin/bash
# GPU round script: tests, smoke, bench variants, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 2560 --warmup 256 --cpu-seconds 8 > gpurun_out/bench_graph.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --mode eager --steps 1024 --no-cpu-baseline > gpurun_out/bench_eager.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --mode rollout --steps 2560 --no-cpu-baseline > gpurun_out/bench_rollout.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1280 --warmup 128 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || exit 1
