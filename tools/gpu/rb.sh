#!/bin/bash
# rBergomi generator on the GPU box: parity tests, bench lines (f64 / f32 normals),
# rocprofv3 kernel-trace summary of the default bench line.
#   gpurun --timeout 900 -- bash tools/gpu/rb.sh <tag>
set -o pipefail
TAG=${1:-rb}
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rbergomi_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload rbergomi --steps 3 --warmup 1 > $O/b_f64.log 2>&1 || { tail -20 $O/b_f64.log; exit 1; }
grep "^{" $O/b_f64.log
timeout -k 10 300 python -u bench.py --workload rbergomi --rb-normals f32 --steps 3 --warmup 1 --no-cpu-baseline > $O/b_f32.log 2>&1 || { tail -20 $O/b_f32.log; exit 1; }
grep "^{" $O/b_f32.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --workload rbergomi --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/b_prof.log 2>&1 || { tail -20 $R/$O/b_prof.log; exit 1; }
grep "^{" $R/$O/b_prof.log
python3 $R/tools/kstats.py $R/$O/prof | head -5
