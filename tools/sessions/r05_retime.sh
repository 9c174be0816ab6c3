#!/bin/bash
# round 5: re-time the config-3 records flagged by tools/sweep_flag.py (timed regions stretched by other workers),
# one K per pass so every worker runs the same kind of launch (the configuration in which the contamination probe,
# tools/sessions/r05_contam.sh, measured 8 workers as clean as one):
#   bash tools/sessions/r05_retime.sh <pairs file> <K list> <budget_s> <workers>
set -u
cd "${GRAFT_REPO_ROOT:-.}"
PAIRS=$1; K=$2; BUDGET=${3:-900}; WORKERS=${4:-8}; NAME=r05_sweep_medium
OUT=gpurun_out/sweep; mkdir -p $OUT
export TMPDIR=/tmp OMP_NUM_THREADS=2
STAMP=$(date +%s)r
timeout -k 10 $((BUDGET + 240)) python -u tools/sweep.py --pairs $PAIRS --k $K --budget $BUDGET \
    --workers $WORKERS --lock-alloc --no-features --check-rows 32 --gold-rows 16 --iters 10 \
    --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP*.jsonl | wc -l; exit $rc
