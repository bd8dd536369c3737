#!/bin/bash
# Round 6: the GPU suite (+ smoke), then the host-API timing (bench.sb3_api with the sb3_loop /
# eval_loop legs) of this tree.
#   gpurun --timeout 900 -- bash tools/gpu/r06_host.sh <tag> [tests|host|all]
set -o pipefail
TAG=${1:-r06}; PHASE=${2:-all}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
if [ "$PHASE" != host ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  echo "[$(date +%T)] smoke"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "$PHASE" != tests ]; then
  echo "[$(date +%T)] host API timing"
  timeout -k 10 400 python -u tools/sb3_time.py --out $O/sb3.jsonl > $O/sb3.log 2>&1 || { tail -20 $O/sb3.log; exit 1; }
  python3 - <<PY
import json
d = json.loads(open("$O/sb3.jsonl").read().splitlines()[-1])
for k in ("vec_env", "vecnorm", "sb3_loop", "eval_loop"):
    print(k, {n: (v["us_median"] if "us_median" in v else v) for n, v in d[k].items()})
for k in ("sb3_loop", "eval_loop"):
    print(k, "pass/floor", {n: (v["us_info_pass"], v["pass_floor_us"], v["us_step_wait"]) for n, v in d[k].items()})
print("single", d["single_env"]["steps_per_s"])
PY
fi
echo "[$(date +%T)] done"
