#!/bin/bash
# Round 3 step 3: the default bench with the time-based warm-up, the same command under
# rocprofv3 --kernel-trace --stats, the he_step launch floors (tools/floor) and the role
# timing of lds_rollout_kernel (-DHE_LDS_TIMING build).
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s3.sh <tag>
set -o pipefail
TAG=${1:-s3}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] bench default"
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log > $O/bench.jsonl
echo "[$(date +%T)] bench under rocprofv3 --kernel-trace --stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-pmc --no-cpu-baseline > $O/bench_rocprof.log 2>&1 || { tail -20 $O/bench_rocprof.log; exit 1; }
cd $R
grep "^{" $O/bench_rocprof.log > $O/bench_under_rocprof.jsonl
echo "[$(date +%T)] he_step floors"
timeout -k 10 120 python -u tools/floor/run.py > $O/floor.json 2>&1 || { tail -20 $O/floor.json; exit 1; }
tail -1 $O/floor.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/floorprof -o run -- python3 $R/tools/floor/run.py > $O/floor_rocprof.log 2>&1 || { tail -20 $O/floor_rocprof.log; exit 1; }
cd $R
echo "[$(date +%T)] role timing"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 2 > $O/lds_timing_2.log 2>&1 || { tail -20 $O/lds_timing_2.log; exit 1; }
cat $O/lds_timing_2.log | grep -v amdgpu.ids
python3 - <<PY
import json, glob, csv
for f in ("bench.jsonl", "bench_under_rocprof.jsonl"):
    for l in open("$O/" + f):
        d = json.loads(l); r = d["roofline"]; s = d.get("step_api") or {}
        print(f, "%.4g" % d["value"], "warmup", d["warmup"], r["kernel_us"], r.get("kernel_us_probe"), r["frac"], "step_api", s.get("kernel_us"), s.get("frac"))
for p in ("prof", "floorprof"):
    for fn in glob.glob("$O/" + p + "/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            print(p, row["Name"][:60], row["Calls"], "%.2f us" % (float(row["AverageNs"]) / 1e3), "min %.2f" % (float(row["MinNs"]) / 1e3))
PY
echo "[$(date +%T)] done"
