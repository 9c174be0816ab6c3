#!/bin/bash
# round 5, session e: (1) software-pipelined row kernel (tuning build: U = -8 / -16) against the shipped U = 16 on
# dense and gather-bound lines, same process, interleaved; (2) PMC of the matrix-core tile kernel (policy / 6-slot ring)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05e; mkdir -p $OUT
export TMPDIR=/tmp
export SPMM_HIP_TUNE_TILES=-1
i=0
for G in "445906 445906 100 33.3333 normal random 0.05 0 0.95 0.05 14" "111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14" \
         "196651 196651 500 166.6667 normal random 0.3 0 0.95 0.05 14" "1248014 1248014 100 33.3333 normal random 0.6 0 0.95 0.05 14" \
         "6158235 6158235 20 6.6667 normal random 0.05 0 0.95 0.05 14" "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"; do
  timeout -k 10 300 python -u tools/tune_kernel.py --gen "$G" --variants "16,1,0,1;-8,1,0,1;-16,1,0,1" --rounds 5 --iters 10 \
      > $OUT/tune_$i.log 2>&1; rc=$?; tail -n 1 $OUT/tune_$i.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
unset SPMM_HIP_TUNE_TILES
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;196651 196651 500 166.6667 normal random 0.3 0 0.5 0.95 14"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pa --output-format csv -o pa -- \
  python3 -u tools/mfma_engine_trace.py --lines "$L" --k 32,128 --launches 5 --plans "policy:;r6:SPMM_HIP_MFMA_RING=6" \
  > $OUT/pa.log 2>&1; rc=$?; tail -n 2 $OUT/pa.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum \
  TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum -d $OUT/pb --output-format csv -o pb -- \
  python3 -u tools/mfma_engine_trace.py --lines "$L" --k 32,128 --launches 5 --plans "policy:;r6:SPMM_HIP_MFMA_RING=6" \
  > $OUT/pb.log 2>&1; rc=$?; tail -n 2 $OUT/pb.log | cut -c1-200; exit $rc
