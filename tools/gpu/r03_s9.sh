#!/bin/bash
# Round 3 step 9: the replay LDS kernel -- its parity tests first, then the GPU suite, bench
# config 6 on lds_replay_kernel against the step_kernel path (HE_LDS_ROLLOUT=0), then the
# reward-priority A/B of step 8.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s9.sh <tag>
set -o pipefail
TAG=${1:-s9}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] replay LDS parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lds_replay or replay_slice or replay_matches" --timeout 200 --timeout-method thread > $O/pytest_replay.log 2>&1 \
  || { echo "replay parity failed"; grep -E "FAIL|Error|assert" $O/pytest_replay.log | head -30; tail -40 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
echo "[$(date +%T)] suite"
bash tools/gpu/tests.sh $TAG || exit 1
for rep in 1 2; do
  for l in 1 0; do
    HE_LDS_ROLLOUT=$l timeout -k 10 300 python -u bench.py --config 6 --no-pmc --no-cpu-baseline --no-step-api > $O/b6_lds${l}_$rep.log 2>&1 || { tail -5 $O/b6_lds${l}_$rep.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1], '%.4g'%d['value'], d['roofline']['kernel_us'], d['roofline']['frac'])
" $O/b6_lds${l}_$rep.log
  done
done
echo "[$(date +%T)] rocprof config 6"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof6 -o run -- python3 bench.py --config 6 --no-pmc --no-cpu-baseline --no-step-api > $O/prof6.log 2>&1 || { tail -5 $O/prof6.log; exit 1; }
find $O/prof6 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/cfg6_kernel_stats.csv
head -4 $O/cfg6_kernel_stats.csv | cut -c1-200
bash tools/gpu/ab_head.sh $TAG 2 pC pD pE pH || exit 1
echo "[$(date +%T)] done"
