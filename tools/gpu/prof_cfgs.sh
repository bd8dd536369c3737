set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-prof_cfgs}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for c in 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg$c -o run -- python3 $R/bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api > $O/bench_cfg${c}_rocprof.log 2>&1 || { tail -20 $O/bench_cfg${c}_rocprof.log; exit 1; }
  grep "^{" $O/bench_cfg${c}_rocprof.log > $O/bench_cfg${c}_under_rocprof.jsonl
  python3 $R/tools/kstats.py $O/prof_cfg$c | head -3
done
