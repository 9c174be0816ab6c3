#!/bin/bash
# round 6, session i: paired short rows -- parity first, then the A/B against the unpaired kernel on
# the avg-5 / avg-10 dataset lines (tools/r06_short_lines.txt), K 8 / 32 / 128, same process, interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_short_lines.txt)" \
    --k 8,32,128 --plans "off:SPMM_HIP_PAIR=-1;on:SPMM_HIP_PAIR=1" --launches 10 --repeat 2 \
    > $OUT/pair_ab.jsonl 2> $OUT/pair_ab.err
rc=$?; wc -l $OUT/pair_ab.jsonl; exit $rc
