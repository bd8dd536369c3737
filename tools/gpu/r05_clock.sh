#!/bin/bash
# Round 5: the -m gpu suite on this tree, the eager / graph device times of the auxiliary
# paths (tools/aux_time.py), the host-API timing, then the role timing with the shader clock of
# the given timing builds (config 2).
#   gpurun --timeout 1200 -- bash tools/gpu/r05_clock.sh <tag> "<timing variants>"
set -o pipefail
TAG=${1:-clk}; TV=${2:-"timing timing_lagxor"}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo "[$(date +%T)] aux_time"
timeout -k 10 300 python -u tools/aux_time.py > $O/aux_time.log 2>&1 || { tail -20 $O/aux_time.log; exit 1; }
grep -v amdgpu.ids $O/aux_time.log
echo "[$(date +%T)] host API"
timeout -k 10 240 python -u tools/sb3_time.py --out $O/sb3.jsonl > $O/sb3.log 2>&1 || { tail -20 $O/sb3.log; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/sb3.jsonl').readline())
print({k: (v['us_per_step'], v['us_median']) for k, v in d['vec_env'].items()}, {k: (v['us_per_step'], v['us_median']) for k, v in d['vecnorm'].items()}, d['single_env']['steps_per_s'])"
for rep in 1 2; do
for v in $TV; do
  echo "[$(date +%T)] role timing $v config 2 ($rep)"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python -u tools/lds_timing.py 65536 256 2 > $O/roles_${v}_cfg2_$rep.log 2>&1 || { tail -5 $O/roles_${v}_cfg2_$rep.log; exit 1; }
  grep -v amdgpu.ids $O/roles_${v}_cfg2_$rep.log
done
done
echo "[$(date +%T)] done"
