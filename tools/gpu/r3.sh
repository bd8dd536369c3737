#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 2560 --warmup 256 --no-cpu-baseline --no-pmc > gpurun_out/b_graph.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode rollout --steps 2560 --no-cpu-baseline --no-pmc > gpurun_out/b_rollout.log 2>&1 || exit 1
CANTORRL_NO_PREFETCH=1 timeout -k 10 300 python bench.py --steps 2560 --warmup 256 --no-cpu-baseline --no-pmc > gpurun_out/b_graph_nopf.log 2>&1 || exit 1
CANTORRL_NO_PREFETCH=1 timeout -k 10 300 python bench.py --mode rollout --steps 2560 --no-cpu-baseline --no-pmc > gpurun_out/b_rollout_nopf.log 2>&1 || exit 1
