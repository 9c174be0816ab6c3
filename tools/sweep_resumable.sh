#!/bin/bash
# Medium dataset (all 16,190 lines) x K in {1,8,32,128}, resumable across gpurun calls, one engine build:
#   bash tools/sweep_resumable.sh <budget_s> <name> [k list] [host workers]
# Lines go in an interleaved order (every 16th line first, then the offsets 8, 4, 12, ...), so a partial sweep still
# covers every class evenly.  profiles/<name>.done (dataset indices already swept; written by tools/sweep_merge.py
# from the merged records -- small, it travels with the tree) is skipped; new records land in
# gpurun_out/sweep/<name>.<stamp>[.w<i>].jsonl, and the call stops starting matrices after <budget_s>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BUDGET=${1:-1000}; NAME=${2:-r03_sweep_medium}; KS=${3:-1,8,32,128}; WORKERS=${4:-1}; WHERE=${5:-}
OUT=gpurun_out/sweep
mkdir -p $OUT
STAMP=$(date +%s)
timeout -k 10 $((BUDGET + 170)) python -u tools/sweep.py --order interleave16 --k $KS --budget $BUDGET \
    --workers $WORKERS --done profiles/$NAME.done ${WHERE:+--where $WHERE} --out $OUT/$NAME.$STAMP.jsonl > $OUT/$NAME.$STAMP.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.$STAMP.log | cut -c1-200; cat $OUT/$NAME.$STAMP*.jsonl | wc -l; exit $rc
