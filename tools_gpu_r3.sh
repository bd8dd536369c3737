#!/bin/bash
# bench variants: prefetch on/off, graph/rollout
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 2560 --warmup 256 --no-cpu-baseline --no-pmc > gpurun_out/b_graph.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode rollout --steps 2560 --no-cpu-baseline --no-pmc > gpurun_out/b_rollout.log 2>&1 || exit 1
CANTORRL_NO_PREFETCH=1 timeout -k 10 300 python bench.py --steps 2560 --warmup 256 --no-cpu-baseline --no-pmc > gpurun_out/b_graph_nopf.log 2>&1 || exit 1
