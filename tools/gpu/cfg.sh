#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
show() { grep "^{" $1 | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$1 value %.4e dev_us/step %.3f kernel_us %.3f frac %.3f mkt/64 %s traffic %s' % (d['value'], 1e3*d['device_ms_per_step'], r['kernel_us'], r['frac'], r.get('market_kernel_us_per_64_steps'), r.get('traffic')))"; }
timeout -k 10 300 python bench.py --config 3 --steps 640 --warmup 128 --no-cpu-baseline > gpurun_out/c3_graph.log 2>&1 || exit 1; show gpurun_out/c3_graph.log
timeout -k 10 300 python bench.py --config 3 --mode rollout --steps 640 --warmup 128 --no-cpu-baseline > gpurun_out/c3_roll.log 2>&1 || exit 1; show gpurun_out/c3_roll.log
timeout -k 10 300 python bench.py --config 5 --steps 1280 --warmup 128 --no-cpu-baseline --no-pmc > gpurun_out/c5_graph.log 2>&1 || exit 1; show gpurun_out/c5_graph.log
timeout -k 10 300 python bench.py --config 2 --steps 2560 --warmup 256 --cpu-seconds 6 > gpurun_out/c2_graph.log 2>&1 || exit 1; show gpurun_out/c2_graph.log
