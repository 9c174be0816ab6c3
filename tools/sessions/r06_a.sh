#!/bin/bash
# round 6, session a: the restructured bench line (medium dataset as the value, config 2 / config 4 sub-records) --
# its GPU tests, then the driver's own command.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06a; mkdir -p $OUT
export TMPDIR=/tmp SPMM_TEST_LOGDIR=$OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 600 --timeout-method thread \
    > $OUT/pytest_bench.log 2>&1
rc=$?; tail -n 8 $OUT/pytest_bench.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc2=$?; tail -c 600 $OUT/bench.json; exit $((rc > rc2 ? rc : rc2))
