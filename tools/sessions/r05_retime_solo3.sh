#!/bin/bash
# round 5: re-time, with ONE worker (no other process on the GPU), the K=32 and K=128 records that still ran > 1.05x the same
# plan in round 3 after the 8-worker re-time, largest excess first (tools/r05_retime_pairs5.txt; pairs3 and pairs4 are done)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
NAME=r05_sweep_medium; OUT=gpurun_out/sweep; mkdir -p $OUT
export TMPDIR=/tmp OMP_NUM_THREADS=16
STAMP=$(date +%s)u
timeout -k 10 1080 python -u tools/sweep.py --pairs tools/r05_retime_pairs5.txt --k 32,128 --budget 840 --batches 3 \
    --no-features --check-rows 32 --gold-rows 16 --iters 10 --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP.jsonl | wc -l; exit $rc
