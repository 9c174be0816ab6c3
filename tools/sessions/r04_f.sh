#!/bin/bash
# round 4, session f: range check beside the tiles + fix-up kernel -- GPU tests, kernel trace,
# then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04f2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_tiles.py tests/test_gpu_policies.py -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt --output-format csv -o kt -- python3 -u tools/mfma_engine_trace.py --k 32,128 \
  --plans "policy:;forced:SPMM_HIP_MFMA=1;np1:SPMM_HIP_MFMA=1,SPMM_HIP_MFMA_NP=1;off:SPMM_HIP_MFMA=-1" \
  > $OUT/kt.log 2>&1; rc=$?; tail -n 8 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_gpu.log; exit $rc
