#!/bin/bash
# Round 3 measurement pass on the final tree: the GPU suite + smoke, then the bench lines
# (headline with PMC + CPU baseline + step API, rocprof of configs 2 and 6, configs 3-6, the
# --gpus 2 rehearsal).
#   gpurun --timeout 1200 -- bash tools/gpu/r03_final.sh <tag>
set -o pipefail
TAG=${1:-final}
bash tools/gpu/round.sh $TAG tests || exit 1
bash tools/gpu/round.sh $TAG bench || exit 1
