#!/bin/bash
# Round 6: the he_step_signal checks and timings: the probe, the host-API tests, the host step
# timing and the bench's sb3_api leg.
#   gpurun --timeout 600 -- bash tools/gpu/r06_signal.sh <tag>
set -o pipefail
TAG=${1:-r06sig}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] probe"
timeout -k 10 60 ./tools/probe/flag_wait 3000 0 > $O/flag_probe.txt 2>&1 || { cat $O/flag_probe.txt; exit 1; }
cat $O/flag_probe.txt
echo "[$(date +%T)] host API tests"
timeout -k 10 300 python -u -m pytest tests/test_host_api_gpu.py tests/test_gpu_single_env.py tests/test_monitor_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_host.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest_host.log | head -30; tail -30 $O/pytest_host.log; exit 1; }
tail -2 $O/pytest_host.log
echo "[$(date +%T)] host step timing"
timeout -k 10 200 python -u tools/host_step_timing.py > $O/host_step.txt 2>&1 || { tail -20 $O/host_step.txt; exit 1; }
cat $O/host_step.txt
echo "[$(date +%T)] sb3 timing"
timeout -k 10 400 python -u tools/sb3_time.py --out $O/sb3.jsonl > $O/sb3.log 2>&1 || { tail -20 $O/sb3.log; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$O/sb3.jsonl").read().splitlines()[-1])
for k in ("vec_env", "sb3_loop"):
    print(k, {n: (v["us_median"] if "us_median" in v else v) for n, v in d[k].items()})
print("single", d["single_env"]["steps_per_s"])
PY
echo "[$(date +%T)] done"
