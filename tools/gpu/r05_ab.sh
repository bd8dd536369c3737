#!/bin/bash
# Round 5: the -m gpu suite, the host-API A/B (round-4 Python package vs this tree), then
# same-box A/B of this tree's library against tools/ab/<variant>.so on the given configs
# (two repetitions, alternating), and the given configs' bench lines with the PMC passes.
#   gpurun --timeout 1200 -- bash tools/gpu/r05_ab.sh <tag> "<ab configs>" "<pmc configs>" <variant>...
set -o pipefail
TAG=${1:-r05ab}; CFGS=${2:-"2 6"}; PMCC=${3:-"6"}; shift 3
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
if [ -z "$NO_SB3" ]; then
for k in 1 2; do
  echo "[$(date +%T)] host API A/B ($k)"
  timeout -k 10 240 python -u tools/sb3_time.py --pkg tools/ab/r04_host --out $O/sb3_ab.jsonl > $O/sb3_old$k.log 2>&1 || { tail -20 $O/sb3_old$k.log; exit 1; }
  timeout -k 10 240 python -u tools/sb3_time.py --out $O/sb3_ab.jsonl > $O/sb3_new$k.log 2>&1 || { tail -20 $O/sb3_new$k.log; exit 1; }
done
python3 - <<PY
import json
for l in open("$O/sb3_ab.jsonl"):
    d = json.loads(l)
    print(d["package"][-40:], {k: (v["us_per_step"], v["us_median"]) for k, v in d["vec_env"].items()},
          {k: (v["us_per_step"], v["us_median"]) for k, v in d["vecnorm"].items()}, d["single_env"]["steps_per_s"])
PY
fi
for c in $CFGS; do
  for rep in 1 2; do
    for v in base "$@"; do
      lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
      CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api --no-sb3-api > $O/b${c}_${v}_$rep.log 2>&1 || { tail -5 $O/b${c}_${v}_$rep.log; exit 1; }
      python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1].split('/')[-1], '%.4g'%d['value'], d['roofline']['kernel_us'], (d.get('shard_check') or {}).get('result'))
" $O/b${c}_${v}_$rep.log
    done
  done
done
for c in $PMCC; do
  echo "[$(date +%T)] bench config $c with PMC passes"
  timeout -k 10 500 python -u bench.py --config $c --no-cpu-baseline --no-sb3-api > $O/bp$c.log 2>&1 || { tail -20 $O/bp$c.log; exit 1; }
  grep "^{" $O/bp$c.log >> $O/bench_pmc.jsonl
  python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; print('cfg', sys.argv[2], '%.4g'%d['value'], r['kernel_us'], r.get('frac'), r.get('traffic_over_bytes'), json.dumps(d.get('step_api'))[:400])
" $O/bp$c.log $c
done
echo "[$(date +%T)] done"
