#!/bin/bash
# Round 5: book pricer skip of options expired on the whole wave -- book/Heston parity tests,
# same-box A/B against the previous library (tools/ab/prevbook.so) on configs 4 / 5
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-book}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "book or heston or full_size_slice or sharding" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
REPS=${REPS:-2} bash tools/gpu/r05_ab3.sh ${1:-book} "" "4 5" prevbook
