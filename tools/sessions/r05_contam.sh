#!/bin/bash
# round 5: is the 8-worker sweep's K=128 timing of big lines contaminated by the other workers?  16 lines (12 that
# ran ~2x slower than in r03 with the same plan, 4 typical), K=128, four ways in a row: 8 workers as the sweep ran;
# 8 workers with 2 hardware queues each (GPU_MAX_HW_QUEUES=2: 16 queues, no HWS oversubscription); 8 workers with
# --lock-alloc (A upload, B/C allocation + fill and the frees under the GPU lock); 6 workers; 1 worker
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/contam; mkdir -p $OUT
export TMPDIR=/tmp OMP_NUM_THREADS=2
COMMON="--dataset tools/r05_contam_lines.txt --k 128 --no-features --check-rows 8 --gold-rows 4 --iters 10"
timeout -k 10 300 python -u tools/sweep.py $COMMON --workers 8 --out $OUT/w8.jsonl > $OUT/w8.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -u tools/sweep.py $COMMON --workers 8 --out $OUT/w8q2.jsonl > $OUT/w8q2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sweep.py $COMMON --workers 6 --out $OUT/w6.jsonl > $OUT/w6.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sweep.py $COMMON --workers 8 --lock-alloc --out $OUT/w8lock.jsonl > $OUT/w8lock.log 2>&1 || exit $?
OMP_NUM_THREADS=16 timeout -k 10 400 python -u tools/sweep.py $COMMON --batches 3 --out $OUT/w1.jsonl > $OUT/w1.log 2>&1
echo rc=$?
