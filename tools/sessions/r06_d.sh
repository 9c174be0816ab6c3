#!/bin/bash
# round 6, session d: packed short rows -- GPU parity (new tests + the parity suite), then an A/B of
# forced packing against none on the avg-5/10/20 lines of the stride-160 sample at K 8 / 32 / 128.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 5 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_short_lines.txt)" \
    --k 8,32,128 --plans "off:SPMM_HIP_PACK=-1;on:SPMM_HIP_PACK=1" --launches 10 > $OUT/ab.jsonl 2> $OUT/ab.err
rc=$?; wc -l $OUT/ab.jsonl; exit $rc
