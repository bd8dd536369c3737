#!/bin/bash
# Round 3 step 44: the UO powers A/B (r03_s43.sh), then the measurement pass of the tree
# (round.sh tests + bench).   gpurun --timeout 1200 -- bash tools/gpu/r03_s44.sh <tag>
set -o pipefail
TAG=${1:-s44}
bash tools/gpu/r03_s43.sh $TAG || exit 1
bash tools/gpu/round.sh $TAG tests || exit 1
bash tools/gpu/round.sh $TAG bench || exit 1
