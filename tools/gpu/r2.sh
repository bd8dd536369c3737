#!/bin/bash
# GPU script: tests, bench (exact kernel timing + PMC traffic), SQ counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 480 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 2560 --warmup 256 --cpu-seconds 8 > gpurun_out/bench_graph.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --mode rollout --steps 2560 --no-cpu-baseline > gpurun_out/bench_rollout.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_sq -o sq -- python3 $R/bench.py --probe > $R/gpurun_out/pmc_sq.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 1280 --warmup 128 --no-cpu-baseline --no-pmc > $R/gpurun_out/prof_bench.log 2>&1 || exit 1
