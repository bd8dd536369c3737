#!/bin/bash
# Dynamic instruction mix + issue utilisation of the headline kernel: four --pmc passes of
# `bench.py --probe` (8 launches), each pass its own run (MI355X_MICROARCH.md PMC slots).
#   gpurun -- bash tools/gpu/pmc.sh <tag> [bench args]
set -o pipefail
TAG=${1:-pmc}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/bench.py --probe $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/a -o a -- $P > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH --output-format csv -d $O/b -o b -- $P > $O/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_WAIT_INST_LDS --output-format csv -d $O/c -o c -- $P > $O/c.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/d -o d -- $P > $O/d.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $O/a $O/b $O/c $O/d
