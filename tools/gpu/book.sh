#!/bin/bash
# book path: GPU parity (book + policy tests), then bench configs 4 and 5
set -o pipefail
TAG=${1:-book}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-step-api --no-pmc > $O/b_cfg$c.log 2>&1 || { tail -20 $O/b_cfg$c.log; exit 1; }
  grep "^{" $O/b_cfg$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['config_index'], '%.3g'%d['value'], r['kernel_us'], r['frac'], r['market_kernel_us_per_64_steps'])"
done
