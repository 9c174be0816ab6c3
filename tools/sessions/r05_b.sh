#!/bin/bash
# round 5, session b: union columns staged through LDS in the matrix-core tile kernel (no premature vmcnt waits) and
# the 6-slot B-operand ring -- bit-exactness tests, then per-kernel times on the probe lines (K 32 / 128)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_tiles.py -x -q \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
LINES="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14;111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14;222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14;196651 196651 500 166.6667 normal random 0.3 0 0.5 0.95 14"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt --output-format csv -o kt -- python3 -u tools/mfma_engine_trace.py \
  --lines "$LINES" --k 32,128 --launches 20 \
  --plans "policy:;r6:SPMM_HIP_MFMA_RING=6;np1:SPMM_HIP_MFMA_NP=1;np1r6:SPMM_HIP_MFMA_NP=1,SPMM_HIP_MFMA_RING=6;off:SPMM_HIP_MFMA=-1" > $OUT/kt.log 2>&1; rc=$?; tail -n 3 $OUT/kt.log | cut -c1-300; exit $rc
