#!/bin/bash
# round 5: why the staged-rows kernel is slow -- kernel trace + two PMC passes on three lines (K 8 / 32), staged
# rows forced vs the row kernel
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/stgdiag; mkdir -p $OUT
export TMPDIR=/tmp
LINES="3483 3483 100 33.3333 normal random 0.3 100 0.05 0.5 14;5588 5588 500 166.6667 normal random 0.05 0 0.95 0.5 14;137518 137518 20 6.6667 normal random 0.05 100 0.95 0.5 14"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $ROOT/tools/mfma_engine_trace.py --lines "$LINES" --k 8,32 --plans "stg:SPMM_HIP_STAGED=1,SPMM_HIP_TILES=-1;rows:SPMM_HIP_STAGED=-1" --launches 5 > $OUT/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pa -o run -- python3 $ROOT/tools/mfma_engine_trace.py --lines "$LINES" --k 8,32 --plans "stg:SPMM_HIP_STAGED=1,SPMM_HIP_TILES=-1;rows:SPMM_HIP_STAGED=-1" --launches 2 > $OUT/pa.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACCUM_PREV_HIRES TCP_TCC_READ_REQ_sum TCC_HIT_sum --output-format csv -d $OUT/pb -o run -- python3 $ROOT/tools/mfma_engine_trace.py --lines "$LINES" --k 8,32 --plans "stg:SPMM_HIP_STAGED=1,SPMM_HIP_TILES=-1;rows:SPMM_HIP_STAGED=-1" --launches 2 > $OUT/pb.log 2>&1
echo pmc rc=$?
