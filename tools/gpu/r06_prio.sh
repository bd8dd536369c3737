#!/bin/bash
# Round 6: the book producers' progress-driven priority (HE_BOOK_PRIO_DYN) against the static
# alternation: same-box A/B on configs 5 and 4, then role timing of both builds.
#   gpurun --timeout 900 -- bash tools/gpu/r06_prio.sh <tag>
set -o pipefail
TAG=${1:-r06prio}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu/ab_head.sh $TAG 5 dyn || exit 1
bash tools/gpu/ab_head.sh $TAG 4 dyn || exit 1
for v in timing timing_dyn; do
  for c in "131072 256 5" "524288 256 4"; do
    echo "== $v $c"
    CANTORRL_HEDGEENV_LIB=$R/tools/abt/$v.so timeout -k 10 120 python tools/lds_timing.py $c > $O/role_${v}_${c// /_}.log 2>&1 || { tail -5 $O/role_${v}_${c// /_}.log; exit 1; }
    cat $O/role_${v}_${c// /_}.log
  done
done
