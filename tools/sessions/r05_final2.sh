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
# human_gene1 fp32 took 2.41 ms in r05bc against 0.363 ms in r05 twins (same engine): five fresh handles, 20 launches
HG="22283 22283 1107.1060000898 1409.1216061190 normal random 0.9314766643 6.1709484000 0.4822844822 0.2820630004 14"
timeout -k 10 300 python -u tools/mfma_engine_trace.py --lines "$HG" --k 32 --dtype f32 --plans "pol:" --repeat 5 --launches 20 > $OUT/human_gene1_f32.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --workload twins --steps 20 --warmup 3 > $OUT/twins.log 2>&1; rc=$?; grep '^{' $OUT/twins.log | cut -c1-300; exit $rc
