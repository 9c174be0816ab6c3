#!/bin/bash
# Medium dataset at 1/16 (every 16th of the 16,190 parameter lines from --offset, ~1,012 matrices) x K in
# {1,8,32,128}, resumable across gpurun calls: records already in profiles/<name>.part are skipped (the .part copy
# travels with the tree; *.jsonl files do not), each call stops starting matrices after the budget (seconds).
#   bash tools/sweep_resumable.sh <offset> <budget_s> <name>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OFF=${1:-0}; BUDGET=${2:-1000}; NAME=${3:-r01_sweep_medium_s16_v8}
OUT=gpurun_out/s16
mkdir -p $OUT
[ -f profiles/$NAME.part ] && cp profiles/$NAME.part $OUT/$NAME.jsonl
timeout -k 10 1150 python -u tools/sweep.py --stride 16 --offset $OFF --k 1,8,32,128 --budget $BUDGET \
    --out $OUT/$NAME.jsonl > $OUT/$NAME.log 2>&1
rc=$?; tail -n 2 $OUT/$NAME.log | cut -c1-200; wc -l $OUT/$NAME.jsonl; exit $rc
