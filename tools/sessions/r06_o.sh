#!/bin/bash
# round 6, session o: streamed rows with more gathers in flight per row (spmm_ring_kernel U = 32 and the pipelined
# row) -- parity of every mode, then the row kernel against ring modes 1 / 2 / 3 on the avg-100/500 lines
# that take no tiles (tools/r06_ring_u_lines.txt), K 32 / 8, same process, interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_ring_u_lines.txt)" \
    --k 32,8 --plans "off:SPMM_HIP_RING=-1;r1:SPMM_HIP_RING=1;r2:SPMM_HIP_RING=2;r3:SPMM_HIP_RING=3" \
    --launches 10 --repeat 2 > $OUT/ring_u_ab.jsonl 2> $OUT/ring_u_ab.err
rc=$?; wc -l $OUT/ring_u_ab.jsonl; exit $rc
