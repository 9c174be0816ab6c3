#!/bin/bash
# round 6, session z: the final build (paired short rows + wide window) -- the whole GPU test suite, the driver's bench command (with the per-matrix
# dataset records) and the same line under rocprofv3 --kernel-trace --stats (no CPU leg).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06z; mkdir -p $OUT
export TMPDIR=/tmp SPMM_TEST_LOGDIR=$OUT/testlogs
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --dataset-out $OUT/ds.jsonl > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -c 300 $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt --output-format csv -o kt -- \
    python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --dataset-out $OUT/ds_prof.jsonl \
    > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?; exit $rc
