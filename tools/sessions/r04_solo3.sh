#!/bin/bash
# round 4: the changed pairs no solo run has timed yet, timed by ONE worker
# (no other process on the GPU), every 16th dataset line first
set -u
cd "${GRAFT_REPO_ROOT:-.}"
BUDGET=${1:-1000}; NAME=r04_ab_solo
OUT=gpurun_out/sweep; mkdir -p $OUT
export TMPDIR=/tmp
STAMP=$(date +%s)
timeout -k 10 $((BUDGET + 170)) python -u tools/sweep.py --order interleave16 --k 32,128 --budget $BUDGET --batches 3 \
    --pairs profiles/r04/solo_rest_pairs.txt --skip-pairs profiles/r04/solo_done_pairs.txt --base-env SPMM_HIP_MFMA=-1 --no-features --check-rows 64 --iters 10 \
    --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP*.jsonl | wc -l; exit $rc
