#!/bin/bash
# round 4: the medium-dataset lines whose plan the shipped engine changes (census: matrix-core tiles), A/B against
# the plan without matrix-core tiles in the same process, resumable across calls:
#   bash tools/sessions/r04_sweep.sh <budget_s> <workers>
set -u
cd "${GRAFT_REPO_ROOT:-.}"
BUDGET=${1:-1000}; WORKERS=${2:-8}; NAME=r04_ab_changed
OUT=gpurun_out/sweep; mkdir -p $OUT
export TMPDIR=/tmp
STAMP=$(date +%s)
timeout -k 10 $((BUDGET + 170)) python -u tools/sweep.py --order interleave16 --k 32,128 --budget $BUDGET \
    --workers $WORKERS --pairs profiles/r04/changed_pairs.txt --base-env SPMM_HIP_MFMA=-1 --no-features --check-rows 64 --iters 10 \
    --skip-pairs profiles/r04/ab_done_pairs.txt --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP*.jsonl | wc -l; exit $rc
