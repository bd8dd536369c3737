#!/bin/bash
# Round 6: policy rollouts on the LDS kernel (lds_rollout_kernel<..., POL>): parity against the
# tile kernels and the host policy restatement, then device time against he_rollout and the tile path.
#   gpurun --timeout 900 -- bash tools/gpu/r06_pol.sh <tag>
set -o pipefail
TAG=${1:-r06pol}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] policy parity"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_kernel_meta_cpu.py -x -v -k "policy or replay or spill" --timeout 120 --timeout-method thread > $O/pytest_pol.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/pytest_pol.log | head -30; tail -40 $O/pytest_pol.log; exit 1; }
tail -2 $O/pytest_pol.log
echo "[$(date +%T)] policy timing (LDS, then tile)"
timeout -k 10 200 python -u tools/policy_time.py 65536 256 100 > $O/policy_time_lds.txt 2>&1 || { tail -20 $O/policy_time_lds.txt; exit 1; }
grep -v amdgpu.ids $O/policy_time_lds.txt
HE_LDS_POLICY=0 timeout -k 10 200 python -u tools/policy_time.py 65536 256 100 > $O/policy_time_tile.txt 2>&1 || { tail -20 $O/policy_time_tile.txt; exit 1; }
grep -v amdgpu.ids $O/policy_time_tile.txt
timeout -k 10 200 python -u tools/policy_time.py 65536 256 100 replay > $O/policy_time_replay_lds.txt 2>&1 || { tail -20 $O/policy_time_replay_lds.txt; exit 1; }
grep -v amdgpu.ids $O/policy_time_replay_lds.txt
HE_LDS_POLICY=0 timeout -k 10 200 python -u tools/policy_time.py 65536 256 100 replay > $O/policy_time_replay_tile.txt 2>&1 || { tail -20 $O/policy_time_replay_tile.txt; exit 1; }
grep -v amdgpu.ids $O/policy_time_replay_tile.txt
echo "[$(date +%T)] policy timing under rocprofv3 --kernel-trace --stats"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/policy_time.py 65536 256 100 > $O/policy_rocprof.log 2>&1 || { tail -20 $O/policy_rocprof.log; exit 1; }
cd $R
python3 tools/kstats.py $O/prof > $O/kstats.txt; head -8 $O/kstats.txt
echo "[$(date +%T)] done"
