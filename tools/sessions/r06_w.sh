#!/bin/bash
# round 6, session w: the wide block window (SPMM_HIP_CAP=4096) -- parity, then the default window
# against the wide one on the avg-50/100/500 lines of the stride-80 sample (tools/r06_ring_lines.txt), K 32 / 128
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_widecap.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_ring_lines.txt)" \
    --k 32,128 --plans "off:;cap4k:SPMM_HIP_CAP=4096" --launches 10 --repeat 2 \
    > $OUT/cap_ab.jsonl 2> $OUT/cap_ab.err
rc=$?; wc -l $OUT/cap_ab.jsonl; exit $rc
