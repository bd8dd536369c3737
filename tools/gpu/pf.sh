#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
show() { grep "^{" $1 | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$1 value %.4e dev_us/step %.3f kernel_us %.3f' % (d['value'], 1e3*d['device_ms_per_step'], r['kernel_us']))"; }
for pf in always rollout always rollout; do
  CANTORRL_PREFETCH=$pf timeout -k 10 300 python bench.py --config 3 --steps 640 --warmup 128 --no-cpu-baseline --no-pmc > gpurun_out/pf_$pf.log 2>&1 || exit 1; show gpurun_out/pf_$pf.log
done
for n in 262144 524288; do for pf in always rollout; do
  CANTORRL_PREFETCH=$pf timeout -k 10 300 python bench.py --envs $n --steps 640 --warmup 128 --no-cpu-baseline --no-pmc > gpurun_out/pf_${pf}_$n.log 2>&1 || exit 1; show gpurun_out/pf_${pf}_$n.log
done; done
