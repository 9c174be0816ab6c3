#!/bin/bash
# round 6, session c (verdict r05 item 5): where a small launch's time goes -- per-block stamps of the row kernel
# (diagnostic build) on 20 lines under 1 M nonzeros at K 1 / 32, their kernel trace (launch gaps); then an A/B of
# vector lanes / shorter split length on the small dense lines (< 4 M nonzeros, avg 50-500) at K 1 / 8 / 32.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/small_breakdown.py --k 1,32 > $OUT/breakdown.jsonl 2> $OUT/breakdown.err
rc=$?; tail -n 2 $OUT/breakdown.jsonl | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt --output-format csv -o kt -- \
    python3 -u tools/small_breakdown.py --k 1,32 > $OUT/kt.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_dense_small_lines.txt)" \
    --k 1,8,32 --plans "pol:;l2:SPMM_HIP_LANES=2;l4:SPMM_HIP_LANES=4;t128:SPMM_HIP_SEQ_MAX=128" --launches 20 \
    > $OUT/lanes.jsonl 2> $OUT/lanes.err
rc=$?; wc -l $OUT/lanes.jsonl; exit $rc
