#!/bin/bash
# Round measurements.  Phase "tests": the whole -m gpu suite + smoke().  Phase "bench":
# the headline bench line (PMC traffic + CPU baseline + step API), the same command under
# rocprofv3 --kernel-trace --stats (and config 6's), configs 3-6 (config 3 with its Gym-API
# step line), and the 2-rank rehearsal of the --gpus N launcher (gloo collectives, both ranks
# on this box's one GPU).  Phase "extra": VecNormalize / analytics device times
# (tools/aux_time.py) and their rocprof summary, the rBergomi bench line under rocprof and
# its VALU pass.
#   gpurun --timeout 1200 -- bash tools/gpu/round.sh <tag> tests|bench|extra
set -o pipefail
TAG=${1:-round}; PHASE=${2:-bench}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
if [ "$PHASE" = tests ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  echo "[$(date +%T)] smoke"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -3 $O/smoke.log
  exit 0
fi
if [ "$PHASE" = extra ]; then
  echo "[$(date +%T)] aux_time"
  timeout -k 10 300 python -u tools/aux_time.py > $O/aux_time.log 2>&1 || { tail -20 $O/aux_time.log; exit 1; }
  grep -v amdgpu.ids $O/aux_time.log
  echo "[$(date +%T)] aux_time under rocprofv3 --kernel-trace --stats"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_aux -o aux -- python3 $R/tools/aux_time.py > $O/aux_prof.log 2>&1 || { tail -20 $O/aux_prof.log; exit 1; }
  cd $R
  python3 tools/kstats.py $O/prof_aux > $O/kstats_aux.txt; head -12 $O/kstats_aux.txt
  echo "[$(date +%T)] rbergomi bench under rocprofv3 --kernel-trace --stats"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rbprof -o run -- python3 $R/bench.py --workload rbergomi --steps 3 --warmup 1 > $O/rb_rocprof.log 2>&1 || { tail -20 $O/rb_rocprof.log; exit 1; }
  cd $R
  grep "^{" $O/rb_rocprof.log > $O/rb_bench.jsonl
  python3 tools/kstats.py $O/rbprof > $O/kstats_rb.txt; head -6 $O/kstats_rb.txt
  echo "[$(date +%T)] rbergomi VALU pass"
  bash tools/gpu/rb_pmc.sh $TAG/rbpmc || exit 1
  echo "[$(date +%T)] done"
  exit 0
fi
echo "[$(date +%T)] bench (default: PMC + CPU baseline + step API)"
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log > $O/bench.jsonl
echo "[$(date +%T)] bench under rocprofv3 --kernel-trace --stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-pmc --no-cpu-baseline --no-step-api > $O/bench_rocprof.log 2>&1 || { tail -20 $O/bench_rocprof.log; exit 1; }
cd $R
grep "^{" $O/bench_rocprof.log > $O/bench_under_rocprof.jsonl
python3 tools/kstats.py $O/prof > $O/kstats.txt; head -4 $O/kstats.txt
echo "[$(date +%T)] config 6 under rocprofv3 --kernel-trace --stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof6 -o run -- python3 $R/bench.py --config 6 --no-pmc --no-cpu-baseline --no-step-api > $O/bench6_rocprof.log 2>&1 || { tail -20 $O/bench6_rocprof.log; exit 1; }
cd $R
python3 tools/kstats.py $O/prof6 > $O/kstats6.txt; head -4 $O/kstats6.txt
for c in 3 4 5 6; do
  echo "[$(date +%T)] bench config $c"
  # configs 4, 5 (book / Heston: producer-bound) and 6 (replay) with the PMC passes: traffic + VALU issue
  pmc=--no-pmc; [ $c != 3 ] && pmc=""
  sapi=--no-step-api; [ $c = 3 ] && sapi=""   # config 3: the Gym-API he_step line at 1M envs
  timeout -k 10 400 python -u bench.py --config $c $pmc $sapi --no-cpu-baseline > $O/b_cfg$c.log 2>&1 || { tail -20 $O/b_cfg$c.log; exit 1; }
  grep "^{" $O/b_cfg$c.log >> $O/bench_cfg345.jsonl
done
echo "[$(date +%T)] --gpus 2 rehearsal (gloo, one GPU)"
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --no-pmc --no-cpu-baseline --no-step-api --steps 512 --warmup 256 > $O/b_gpus2.log 2>&1 || { tail -30 $O/b_gpus2.log; exit 1; }
grep "^{" $O/b_gpus2.log > $O/bench_gpus2_rehearsal.jsonl
python3 - <<PY
import json
for f in ("bench.jsonl", "bench_under_rocprof.jsonl", "bench_cfg345.jsonl", "bench_gpus2_rehearsal.jsonl"):
    for l in open("$O/" + f):
        d = json.loads(l); r = d.get("roofline", {})
        print(f, d["config"].get("config_index"), d["n_gpus"], "%.4g" % d["value"], r.get("kernel_us"), r.get("frac"), r.get("traffic_over_bytes"), (r.get("valu") or {}).get("valu_issue_frac"), d.get("gather", {}).get("envs_with_finished_episode"), (d.get("policy_api") or {}).get("kernel_us"))
PY
echo "[$(date +%T)] done"
