#!/bin/bash
# Round 3 step 45: the GPU suite + smoke on the tree with HE_BOOK_EXP_FAST_UO on, and config 5.
#   gpurun --timeout 900 -- bash tools/gpu/r03_s45.sh <tag>
set -o pipefail
TAG=${1:-s45}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/round.sh $TAG tests || exit 1
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --no-step-api > $O/b_cfg5.log 2>&1 || { tail -20 $O/b_cfg5.log; exit 1; }
grep "^{" $O/b_cfg5.log > $O/bench_cfg5.jsonl
python3 -c "
import json
d=json.loads(open('$O/bench_cfg5.jsonl').readline()); r=d['roofline']; print('config 5', '%.4g' % d['value'], r.get('kernel_us'), r.get('frac'), r.get('traffic_over_bytes'))
"
echo "[$(date +%T)] done"
