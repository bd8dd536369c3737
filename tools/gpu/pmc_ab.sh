#!/bin/bash
# PMC passes (one counter group per run) over step_bench for each tools/ab/*.so
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
N=${1:-65536}
G1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU"
G2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32"
G3="GRBM_GUI_ACTIVE GRBM_COUNT"
for l in tools/ab/*.so; do b=$(basename $l .so)
  k=0
  for G in "$G1" "$G2" "$G3"; do k=$((k+1))
    STEP_BENCH_REPS=2 timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmc/$b/g$k -o g -- ./tools/step_bench $N $l > gpurun_out/pmc/${b}_g$k.log 2>&1 || { tail -5 gpurun_out/pmc/${b}_g$k.log; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc/$b
done
