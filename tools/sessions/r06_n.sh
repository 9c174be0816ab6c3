#!/bin/bash
# round 6, session n: streamed rows (spmm_ring_kernel) -- parity first, then forced streaming against
# the row kernel on the avg-50/100/500 lines of the stride-80 sample (tools/r06_ring_lines.txt), K 8 / 32 / 128, same
# process, interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_ring_lines.txt)" \
    --k 32,8,128 --plans "off:SPMM_HIP_RING=-1;on:SPMM_HIP_RING=1" --launches 10 --repeat 2 \
    > $OUT/ring_ab.jsonl 2> $OUT/ring_ab.err
rc=$?; wc -l $OUT/ring_ab.jsonl; exit $rc
