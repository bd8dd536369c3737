#!/bin/bash
# Round 5: replay loader line hand-over -- replay parity tests, same-box A/B against the
# previous loader (tools/ab/prevload.so), the read-traffic counters
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-replay}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "replay" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
REPS=3 bash tools/gpu/r05_ab3.sh ${1:-replay} "" "6" prevload || exit 1
timeout -k 10 900 python -u tools/traffic_calib.py --out $O/traffic > $O/traffic.log 2>&1 || { tail -5 $O/traffic.log; exit 1; }
grep -v amdgpu.ids $O/traffic.log
