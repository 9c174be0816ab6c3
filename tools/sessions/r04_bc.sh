#!/bin/bash
# round 4, sessions b + c in one call: fp32 matrix-core tests, matrix-core kernel PMC, gate fit A/B sample
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04b; mkdir -p $OUT gpurun_out/r04c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
L="39120 39120 500 166.6667 normal random 0.05 0 0.05 0.95 14;196651 196651 500 166.6667 normal random 0.3 0 0.5 0.95 14"
P="np1:SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NP=1;np2:SPMM_HIP_MFMA=2;nochk:SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NP=1,SPMM_HIP_MFMA_CHECK=0"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/mfma_engine_trace.py --lines "$L" --k 32,128 --plans "$P" --launches 5 > $OUT/kt.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d $OUT/p1 -o run --output-format csv -- python3 tools/mfma_engine_trace.py --lines "$L" --k 32,128 --plans "$P" --launches 5 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o run --output-format csv -- python3 tools/mfma_engine_trace.py --lines "$L" --k 32,128 --plans "$P" --launches 5 > $OUT/p2.log 2>&1 || exit $?
grep '^{' $OUT/kt.log | cut -c1-150
OUT=gpurun_out/r04c
timeout -k 10 800 python -u tools/sweep.py --dataset tools/r04_fit_lines.txt --k 32,128 --env SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NPC=96 \
    --base-env SPMM_HIP_MFMA=-1 --workers 6 --budget 640 --check-rows 64 --no-features --iters 10 --order interleave16 \
    --out $OUT/fit_ab.jsonl > $OUT/fit_ab.log 2>&1; rc=$?; tail -n 3 $OUT/fit_ab.log; cat $OUT/fit_ab*.jsonl | wc -l; exit $rc
