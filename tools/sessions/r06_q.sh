#!/bin/bash
# round 6, session q: the shipped library rebuilt after the streamed-row and x-window experiments (sources identical
# to the final build of session m, engine 08e48ee7) -- smoke() and the whole GPU test suite on it; then the per-block
# stamps (diagnostic build) of the avg-100/500 lines that take no tiles at K = 32 (tools/r06_ring_u_lines.txt): where
# the dense classes' launch time goes
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06q; mkdir -p $OUT
export TMPDIR=/tmp SPMM_TEST_LOGDIR=$OUT/testlogs
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -n 2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/small_breakdown.py --lines-file tools/r06_ring_u_lines.txt --k 32 \
    > $OUT/dense_stamps.jsonl 2> $OUT/dense_stamps.err
rc=$?; wc -l $OUT/dense_stamps.jsonl; exit $rc
