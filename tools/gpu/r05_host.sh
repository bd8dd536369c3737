#!/bin/bash
# Round 5, host-path pass: the -m gpu suite + smoke, the SB3 / single-env host-API timing of
# the round-4 Python package (tools/ab/r04_host) against this tree's (same library), then
# the default bench line.
#   gpurun --timeout 1200 -- bash tools/gpu/r05_host.sh <tag>
set -o pipefail
TAG=${1:-r05host}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[$(date +%T)] smoke"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for k in 1 2; do
  echo "[$(date +%T)] host API: round-4 package, then this tree ($k)"
  timeout -k 10 240 python -u tools/sb3_time.py --pkg tools/ab/r04_host --out $O/sb3_ab.jsonl > $O/sb3_old$k.log 2>&1 || { tail -20 $O/sb3_old$k.log; exit 1; }
  timeout -k 10 240 python -u tools/sb3_time.py --out $O/sb3_ab.jsonl > $O/sb3_new$k.log 2>&1 || { tail -20 $O/sb3_new$k.log; exit 1; }
done
python3 - <<PY
import json
for l in open("$O/sb3_ab.jsonl"):
    d = json.loads(l)
    print(d["package"][-30:], {k: v["us_per_step"] for k, v in d["vec_env"].items()},
          {k: v["us_per_step"] for k, v in d["vecnorm"].items()}, d["single_env"]["steps_per_s"])
PY
echo "[$(date +%T)] bench (default)"
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log > $O/bench.jsonl
python3 -c "
import json; d=json.loads(open('$O/bench.jsonl').readline()); r=d['roofline']
print(d['value'], r['kernel_us'], r['frac'], r.get('traffic_over_bytes'))
print(json.dumps(d['step_api'])); print(json.dumps(d['sb3_api']))"
echo "[$(date +%T)] done"
