#!/bin/bash
# round 4 final build, part 2: the default bench line under rocprofv3 (kernel stats), the twins line
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 50 --warmup 10 > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload twins --steps 20 --warmup 3 > $OUT/twins.log 2>&1; rc=$?; grep '^{' $OUT/twins.log | cut -c1-300; exit $rc
