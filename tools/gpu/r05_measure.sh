#!/bin/bash
# Round 5 measurement pass: the host-API timing of this tree, config 3's bench line (its
# Gym-API step at 1M envs with the step kernel's PMC traffic), the rBergomi bench line
# (VALU roofline + traffic from PMC passes), and the wave-state PMC passes of config 4 on
# this tree and on the steppers-idle diagnostic build (tools/ab/diag2.so: HE_LDS_DIAG=2).
#   gpurun --timeout 1200 -- bash tools/gpu/r05_measure.sh <tag>
set -o pipefail
TAG=${1:-meas}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] host API"
timeout -k 10 240 python -u tools/sb3_time.py --out $O/sb3.jsonl > $O/sb3.log 2>&1 || { tail -20 $O/sb3.log; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/sb3.jsonl').readline())
print({k: (v['us_per_step'], v['us_median']) for k, v in d['vec_env'].items()}, {k: (v['us_per_step'], v['us_median']) for k, v in d['vecnorm'].items()}, d['single_env']['steps_per_s'])"
echo "[$(date +%T)] bench config 3 (step_api at 1M envs + PMC)"
timeout -k 10 500 python -u bench.py --config 3 --no-cpu-baseline > $O/b3.log 2>&1 || { tail -20 $O/b3.log; exit 1; }
grep "^{" $O/b3.log > $O/bench_cfg3.jsonl
python3 -c "
import json
d=json.loads(open('$O/bench_cfg3.jsonl').readline()); print('%.4g'%d['value'], d['roofline']['kernel_us'], d['roofline']['frac'], d['roofline'].get('traffic_over_bytes')); print(json.dumps(d['step_api']))"
echo "[$(date +%T)] rbergomi bench (PMC passes)"
timeout -k 10 500 python -u bench.py --workload rbergomi > $O/rb.log 2>&1 || { tail -20 $O/rb.log; exit 1; }
grep "^{" $O/rb.log > $O/rb_bench.jsonl
python3 -c "
import json
d=json.loads(open('$O/rb_bench.jsonl').readline()); print('%.4g'%d['value'], json.dumps(d['roofline']))"
for v in base diag2; do
  echo "[$(date +%T)] pmc_stall config 4 ($v)"
  lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
  CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 400 python -u tools/pmc_stall.py --config 4 > $O/stall4_$v.log 2>&1 || { tail -5 $O/stall4_$v.log; exit 1; }
  cat $O/stall4_$v.log
done
echo "[$(date +%T)] done"
