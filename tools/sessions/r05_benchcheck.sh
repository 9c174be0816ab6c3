#!/bin/bash
# round 5: the bench line's new oracle check of C (config 2 full matrix + the dataset record's CPU leg) and the twins
# line, on the shipped engine, before the final session
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05bc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --workload twins --steps 10 --warmup 3 > $OUT/twins.log 2>&1; rc=$?; grep '^{' $OUT/twins.log | cut -c1-300; exit $rc
