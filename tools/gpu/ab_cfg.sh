#!/bin/bash
# A/B of libhedgeenv variants (tools/ab/<name>.so) on bench configs, plus rocprof of the
# auxiliary kernels (VecNormalize, analytics):
#   gpurun -- bash tools/gpu/ab_cfg.sh <tag> "<configs>" <variant>...
set -o pipefail
TAG=${1:-ab}; CFGS=${2:-"4 5"}; shift 2
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vecnorm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_vn.log 2>&1 || { tail -30 $O/pytest_vn.log; exit 1; }
tail -1 $O/pytest_vn.log
timeout -k 10 200 python -u tools/aux_time.py > $O/aux_time.log 2>&1 || { tail -20 $O/aux_time.log; exit 1; }
head -8 $O/aux_time.log
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/auxprof -o run -- python3 $R/tools/aux_time.py > $R/$O/aux_prof.log 2>&1) || { tail -20 $O/aux_prof.log; exit 1; }
python3 tools/kstats.py $O/auxprof | grep -E "vn_|step1" || true
for c in $CFGS; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib=$R/tools/ab/$v.so
    CANTORRL_HEDGEENV_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-pmc --no-cpu-baseline --no-step-api --steps 1024 > $O/b${c}_$v.log 2>&1 || { tail -5 $O/b${c}_$v.log; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[1], '%.4g'%d['value'], d['roofline']['kernel_us'])
" $O/b${c}_$v.log
  done
done
if [ -n "$HEADLINE" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench2.log 2>&1 || { tail -5 $O/bench2.log; exit 1; }
  grep "^{" $O/bench2.log > $O/bench2.jsonl
  python3 -c "
import json
d=json.loads(open('$O/bench2.jsonl').readline()); r=d['roofline']; print('%.4g'%d['value'], r['kernel_us'], r['frac'], json.dumps(r.get('valu')))"
fi
