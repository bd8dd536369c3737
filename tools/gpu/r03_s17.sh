#!/bin/bash
# Round 3 step 17: what holds the replay reward stepper (busy ~3,200 cycles per step): role
# timing of config 6 for the default build and diagnostic builds without the reward / done
# stores (d3), with multiplies for its two divisions (d4), without action loads (d5), without
# table reads (d1).
#   gpurun --timeout 600 -- bash tools/gpu/r03_s17.sh <tag>
set -o pipefail
TAG=${1:-s17}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for t in timing timing_d3 timing_d4 timing_d5 timing_d1; do
  echo "[$(date +%T)] role timing config 6 $t"
  CANTORRL_HEDGEENV_LIB=$R/tools/abt/$t.so timeout -k 10 120 python tools/lds_timing.py 65536 256 6 > $O/role6_$t.log 2>&1 || { tail -5 $O/role6_$t.log; exit 1; }
  grep -v amdgpu.ids $O/role6_$t.log
done
echo "[$(date +%T)] done"
