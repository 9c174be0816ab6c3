#!/bin/bash
# round 5: the whole medium dataset (16,190 lines) x K in {1,8,32,128} fp64 on ONE engine build (verdict r04 item 4),
# resumable across calls: profiles/r05_sweep_medium.done (tools/sweep_merge.py) lists the lines already swept.
#   bash tools/sessions/r05_sweep.sh <budget_s> <workers>
# Every record: 10 HIP-event-timed launches after 3 warm-ups (the timed regions of the workers serialised by a lock),
# 32 sampled rows against the oracle (bit-exact on exact rows, 1e-10 normwise + fp128 gold on the rest).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
BUDGET=${1:-900}; WORKERS=${2:-8}; NAME=r05_sweep_medium
OUT=gpurun_out/sweep; mkdir -p $OUT
export TMPDIR=/tmp OMP_NUM_THREADS=${SWEEP_OMP:-2}
STAMP=$(date +%s)
timeout -k 10 $((BUDGET + 240)) python -u tools/sweep.py --order interleave16 --k 1,8,32,128 --budget $BUDGET \
    --workers $WORKERS --lock-alloc --no-features --check-rows 32 --gold-rows 16 --iters 10 --done profiles/$NAME.done \
    --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP*.jsonl | wc -l; exit $rc
