#!/bin/bash
# round 4, session e: the flag/prepass matrix-core kernel -- GPU tests, kernel trace of the prepass and tile kernels,
# then the small-matrix one-launch-panel A/B (session d)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_tiles.py tests/test_gpu_policies.py -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 -u tools/mfma_engine_trace.py --k 32,128 \
  --plans "policy:;forced:SPMM_HIP_MFMA=1;np1:SPMM_HIP_MFMA=1,SPMM_HIP_MFMA_NP=1;off:SPMM_HIP_MFMA=-1" \
  > $OUT/kt.log 2>&1; rc=$?; tail -n 8 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
L=$(paste -sd';' tools/r04_small_lines.txt)
timeout -k 10 600 python -u tools/mfma_ab.py --lines "$L" --k 32,128 --modes "off:SPMM_HIP_SMALL_KW=0;kw16:SPMM_HIP_SMALL_KW=16;kw8:SPMM_HIP_SMALL_KW=8" --budget 480 > $OUT/ab_small.jsonl 2> $OUT/ab_small.err; rc=$?; wc -l $OUT/ab_small.jsonl; exit $rc
