#!/bin/bash
# Medium dataset at 1/16 (every 16th of the 16,190 parameter lines = 1,012 matrices) x K in {1,8,32,128}, resumable:
# records already in profiles/r01_sweep_medium_s16_v8.jsonl are skipped; each call stops starting matrices after
# --budget seconds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s16
mkdir -p $OUT
[ -f profiles/r01_sweep_medium_s16_v8.jsonl ] && cp profiles/r01_sweep_medium_s16_v8.jsonl $OUT/sweep.jsonl
timeout -k 10 1150 python -u tools/sweep.py --stride 16 --k 1,8,32,128 --budget ${1:-1000} --out $OUT/sweep.jsonl \
    > $OUT/sweep.log 2>&1
rc=$?; tail -n 2 $OUT/sweep.log | cut -c1-200; wc -l $OUT/sweep.jsonl; exit $rc
