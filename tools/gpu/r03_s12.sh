#!/bin/bash
# Round 3 step 12: lagged obs stepper (greeks by the reward stepper) in the lean GBM kernel;
# replay steppers with branch-free divisions; VecNormalize with every row input loaded before
# the merge and the fused moments from the he_step workgroup's LDS rows.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s12.sh <tag>
set -o pipefail
TAG=${1:-s12}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] suite"
bash tools/gpu/tests.sh $TAG || exit 1
bash tools/gpu/ab_head.sh $TAG 2 nolag || exit 1
echo "[$(date +%T)] role timing config 2"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 > $O/role_timing2.log 2>&1 || { tail -5 $O/role_timing2.log; exit 1; }
grep -v amdgpu.ids $O/role_timing2.log
bash tools/gpu/ab_head.sh $TAG 6 rD8 rp2 || exit 1
echo "[$(date +%T)] role timing config 6"
CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 120 python tools/lds_timing.py 65536 256 6 > $O/role_timing6.log 2>&1 || { tail -5 $O/role_timing6.log; exit 1; }
grep -v amdgpu.ids $O/role_timing6.log
echo "[$(date +%T)] vecnorm timing"
timeout -k 10 200 python -u tools/aux_time.py > $O/aux_time.log 2>&1 || { tail -20 $O/aux_time.log; exit 1; }
head -8 $O/aux_time.log
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/auxprof -o run -- python3 $R/tools/aux_time.py > $O/aux_prof.log 2>&1) || { tail -20 $O/aux_prof.log; exit 1; }
python3 tools/kstats.py $O/auxprof | grep -E "vn_|step1" || true
echo "[$(date +%T)] done"
