#!/bin/bash
# Round 3 step 4: measurements (tools/gpu/r03_s3.sh) + same-box A/B of the producer variants
# (lock4: whole-block lockstep producers at 4 waves/SIMD; rcp: reciprocal log ratio) on
# configs 2 and 4, and of the replay variants (epw32, pf8) on config 6.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s4.sh <tag>
set -o pipefail
TAG=${1:-s4}
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu/r03_s3.sh $TAG || exit 1
for c in 2 4; do
  echo "[$(date +%T)] A/B config $c"
  bash tools/gpu/ab_head.sh $TAG $c lock4 lock4rcp rcp || exit 1
done
echo "[$(date +%T)] A/B config 6"
bash tools/gpu/ab_head.sh $TAG 6 epw32 pf8 || exit 1
echo "[$(date +%T)] done"
