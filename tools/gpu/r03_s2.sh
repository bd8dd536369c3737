#!/bin/bash
# Round 3 step 2: the whole GPU suite on the new tree, the launch-timing diagnostic, the
# replay bench config and the default bench line.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s2.sh <tag>
set -o pipefail
TAG=${1:-s2}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log; grep -E "RCCL all_gather|us per boundary" $O/pytest_gpu.log | head -3
echo "[$(date +%T)] launch timing config 2"
timeout -k 10 120 python -u tools/launch_timing.py --config 2 > $O/launch_timing_2.json 2>&1 || { tail -20 $O/launch_timing_2.json; exit 1; }
cat $O/launch_timing_2.json
echo "[$(date +%T)] bench config 6 (replay)"
timeout -k 10 300 python -u bench.py --config 6 --no-pmc --no-cpu-baseline > $O/b_cfg6.log 2>&1 || { tail -20 $O/b_cfg6.log; exit 1; }
grep "^{" $O/b_cfg6.log > $O/bench_cfg6.jsonl
echo "[$(date +%T)] bench default"
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log > $O/bench.jsonl
python3 - <<PY
import json
for f in ("bench.jsonl", "bench_cfg6.jsonl"):
    for l in open("$O/" + f):
        d = json.loads(l); r = d["roofline"]; s = d.get("step_api") or {}; c = d.get("cpu_baseline") or {}
        print(f, d["config"]["config_index"], "%.4g" % d["value"], r["kernel_us"], r.get("kernel_us_probe"), r["frac"],
              r.get("traffic_over_bytes"), "step_api", s.get("kernel_us"), s.get("frac"), "cpu", c.get("value"), c.get("single_core_value"))
PY
echo "[$(date +%T)] done"
