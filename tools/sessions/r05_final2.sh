#!/bin/bash
# round 5 final build, part 2: config 2 alone under rocprofv3 (the kernel stats the roofline line follows from,
# verdict r04 item 2), the default bench line (dataset record, CPU baseline, oracle check of C), the twins line
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r05f; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg2 -o run -- python3 $ROOT/bench.py --no-dataset --no-cpu-baseline --no-multi-handle --steps 50 --warmup 10 > $OUT/bench_cfg2_prof.log 2>&1; rc=$?; grep '^{' $OUT/bench_cfg2_prof.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd $ROOT
timeout -k 10 900 python -u bench.py --steps 50 --warmup 10 > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --workload twins --steps 20 --warmup 3 > $OUT/twins.log 2>&1; rc=$?; grep '^{' $OUT/twins.log | cut -c1-300; exit $rc
