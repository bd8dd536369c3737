#!/bin/bash
# Round 6 measurements: host step timing; same-box A/B of this tree's kernels against round 5's
# (tools/ab/r05.so) on the headline; the action footprint (config 2 with 4 action sets =
# 537 MB, past the 256 MB Infinity Cache) against config 3.
#   gpurun --timeout 900 -- bash tools/gpu/r06_measure.sh <tag> [host|ab|mall|all]
set -o pipefail
TAG=${1:-r06m}; PHASE=${2:-all}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
Q="--no-pmc --no-cpu-baseline --no-step-api --no-sb3-api"
line() { python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']
print(sys.argv[1].split('/')[-1], 'value %.4g'%d['value'], 'kernel_us', r.get('kernel_us'), 'frac', r.get('frac'))
" $1; }
if [ "$PHASE" = host ] || [ "$PHASE" = all ] || [ "$PHASE" = scan ]; then
  echo "[$(date +%T)] host step timing"
  timeout -k 10 200 python -u tools/host_step_timing.py > $O/host_step.log 2>&1 || { tail -20 $O/host_step.log; exit 1; }
  grep -v amdgpu.ids $O/host_step.log
fi
if [ "$PHASE" = ab ] || [ "$PHASE" = all ]; then
  for rep in 1 2 3; do
    for v in base r05; do
      lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
      CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py $Q > $O/ab_${v}_$rep.log 2>&1 || { tail -5 $O/ab_${v}_$rep.log; exit 1; }
      line $O/ab_${v}_$rep.log
    done
  done
fi
if [ "$PHASE" = mall ] || [ "$PHASE" = all ]; then
  for a in "--config 2" "--config 2 --action-sets 4" "--config 3" "--config 2" "--config 2 --action-sets 4" "--config 3"; do
    f=$O/mall_$(echo $a | tr -d ' -').log
    timeout -k 10 300 python -u bench.py $Q $a > $f 2>&1 || { tail -5 $f; exit 1; }
    line $f
  done
fi
if [ "$PHASE" = persist ]; then
  echo "[$(date +%T)] parity (LDS / persistent grid / tiny marks)"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lds_rollout or lds_persistent or full_size" --timeout 120 --timeout-method thread > $O/persist_pytest.log 2>&1 || { tail -30 $O/persist_pytest.log; exit 1; }
  tail -1 $O/persist_pytest.log
  for rep in 1 2; do
    for ps in 1 0; do
      f=$O/persist${ps}_cfg3_$rep.log
      HE_LDS_PERSIST=$ps timeout -k 10 300 python -u bench.py $Q --config 3 > $f 2>&1 || { tail -5 $f; exit 1; }
      line $f
    done
    f=$O/persist1_cfg2_$rep.log
    timeout -k 10 300 python -u bench.py $Q --config 2 > $f 2>&1 || { tail -5 $f; exit 1; }
    line $f
  done
fi
if [ "$PHASE" = clock ]; then
  # config 2 over a timed region as long as config 3's (1,600 launches, ~0.43 s) against the default 100
  for rep in 1 2; do
    for st in 25600 409600; do
      f=$O/clock_cfg2_${st}_$rep.log
      timeout -k 10 300 python -u bench.py $Q --config 2 --steps $st > $f 2>&1 || { tail -5 $f; exit 1; }
      line $f
    done
    f=$O/clock_cfg3_$rep.log
    timeout -k 10 300 python -u bench.py $Q --config 3 > $f 2>&1 || { tail -5 $f; exit 1; }
    line $f
  done
fi
if [ "$PHASE" = scan ]; then
  # the per-env-step kernel time against the env count (rounds of workgroups, footprint) and K
  for a in "--envs 65536" "--envs 131072" "--envs 262144" "--envs 524288" "--envs 1048576" "--envs 1048576 --rollout-k 64" "--envs 1048576 --rollout-k 16" "--envs 65536 --rollout-k 64" "--envs 65536 --rollout-k 16" "--envs 2097152"; do
    f=$O/scan_$(echo $a | tr -d ' -').log
    timeout -k 10 300 python -u bench.py $Q --config 2 $a > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; c=d['config']
print(sys.argv[1].split('/')[-1], 'envs', c['envs_per_gpu'], 'K', c['rollout_k'], 'kernel_us %.1f' % r['kernel_us'], 'ns/env-step %.4f' % (r['kernel_us'] * 1e3 / (c['envs_per_gpu'] * c['rollout_k'])), 'frac', r['frac'])
" $f
  done
fi
if [ "$PHASE" = persist45 ]; then
  for rep in 1 2; do
    for c in 4 5; do
      for ps in 1 0; do
        f=$O/persist${ps}_cfg${c}_$rep.log
        HE_LDS_PERSIST=$ps timeout -k 10 300 python -u bench.py $Q --config $c > $f 2>&1 || { tail -5 $f; exit 1; }
        line $f
      done
    done
  done
fi
if [ "$PHASE" = balance ]; then
  echo "[$(date +%T)] parity (LDS / persistent / replay)"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lds or full_size or replay" --timeout 120 --timeout-method thread > $O/bal_pytest.log 2>&1 || { tail -30 $O/bal_pytest.log; exit 1; }
  tail -1 $O/bal_pytest.log
  for c in 3 4 5 2 6 3 4 5; do
    for v in claim_nopersist claim_persist noclaim_nopersist; do
      lib=""; ps=0
      [ $v = claim_persist ] && ps=1
      [ $v = noclaim_nopersist ] && lib=$R/tools/ab/noclaim.so
      f=$O/bal_cfg${c}_$v.log; [ -e $f ] && f=$O/bal_cfg${c}_${v}_2.log
      CANTORRL_HEDGEENV_LIB=$lib HE_LDS_PERSIST=$ps timeout -k 10 300 python -u bench.py $Q --config $c > $f 2>&1 || { tail -5 $f; exit 1; }
      line $f
    done
  done
fi
if [ "$PHASE" = clk ]; then
  # the shader clock the timing build reports (s_memtime per s_memrealtime tick), config 2 and
  # 3 back to back twice, then the plain bench lines of both
  for rep in 1 2; do
    for n in 65536 1048576; do
      echo "== timing build, $n envs (rep $rep)"
      CANTORRL_HEDGEENV_LIB=$R/tools/abt/timing.so timeout -k 10 200 python -u tools/lds_timing.py $n 256 > $O/clk_${n}_$rep.log 2>&1 || { tail -5 $O/clk_${n}_$rep.log; exit 1; }
      grep -v amdgpu.ids $O/clk_${n}_$rep.log | head -8
    done
    for c in 2 3; do
      f=$O/clk_bench_cfg${c}_$rep.log
      timeout -k 10 300 python -u bench.py $Q --config $c > $f 2>&1 || { tail -5 $f; exit 1; }
      line $f
    done
  done
fi
if [ "$PHASE" = book ]; then
  echo "[$(date +%T)] parity (books / Heston)"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_book_cpu.py -x -q -k "book or heston or barrier or full_size" --timeout 120 --timeout-method thread > $O/book_pytest.log 2>&1 || { tail -30 $O/book_pytest.log; exit 1; }
  tail -1 $O/book_pytest.log
  for rep in 1 2 3; do
    for v in base pre_sh; do
      lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
      f=$O/book_cfg5_${v}_$rep.log
      CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py $Q --config 5 > $f 2>&1 || { tail -5 $f; exit 1; }
      line $f
    done
  done
fi
if [ "$PHASE" = rb ] || [ "$PHASE" = all ]; then
  echo "[$(date +%T)] rbergomi tests"
  timeout -k 10 300 python -u -m pytest tests/test_rbergomi_gpu.py -x -q --timeout 120 --timeout-method thread > $O/rb_pytest.log 2>&1 || { tail -30 $O/rb_pytest.log; exit 1; }
  tail -1 $O/rb_pytest.log
  for rep in 1 2; do
    for nm in f64 f32; do
      for valu in 0 1; do
        f=$O/rb_${nm}_valu${valu}_$rep.log
        RB_MC_MFMA=$((1 - valu)) timeout -k 10 300 python -u bench.py --workload rbergomi --rb-normals $nm --no-pmc --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
        python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]
print(sys.argv[1].split('/')[-1], 'options/s %.4g' % d['value'], 'kernel ms', d['kernel']['ms_per_launch'])
" $f
      done
    done
  done
fi
echo "[$(date +%T)] done"
