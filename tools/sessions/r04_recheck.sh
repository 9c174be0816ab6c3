#!/bin/bash
# round 4: the changed-lines A/B pairs that measured below 1.0x with 8 sweep workers sharing the GPU, timed again
# by ONE worker (no other process on the GPU), same interleaved batches -- contention or the plan?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
BUDGET=${1:-900}; NAME=r04_ab_recheck
OUT=gpurun_out/sweep; mkdir -p $OUT
export TMPDIR=/tmp
STAMP=$(date +%s)
timeout -k 10 $((BUDGET + 170)) python -u tools/sweep.py --k 32,128 --budget $BUDGET --batches 3 \
    --pairs profiles/r04/recheck_pairs.txt --base-env SPMM_HIP_MFMA=-1 --no-features --check-rows 16 --iters 10 \
    --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP*.jsonl | wc -l; exit $rc
