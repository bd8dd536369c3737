#!/bin/bash
# Round 5: read-traffic counter calibration (tools/traffic_calib.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-traffic}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u tools/traffic_calib.py --out $O/traffic > $O/traffic.log 2>&1; rc=$?
grep -v amdgpu.ids $O/traffic.log; exit $rc
