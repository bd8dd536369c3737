#!/bin/bash
# Round 3 step 16 = steps 14 + 15 in one call.
#   gpurun --timeout 1200 -- bash tools/gpu/r03_s16.sh <tag>
set -o pipefail
TAG=${1:-s16}
bash tools/gpu/r03_s14.sh $TAG || exit 1
bash tools/gpu/r03_s15.sh $TAG || exit 1
