#!/bin/bash
# round 5, session a: counter list of this pool's gfx950, smoke, config-2-only kernel trace (verdict r04 item 2)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; rc=$?; echo "list rc=$rc"; wc -l $OUT/counters.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o c2 -- \
  python3 -u bench.py --no-dataset --no-cpu-baseline --no-multi-handle --steps 20 --warmup 5 > $OUT/c2.log 2>&1; rc=$?; tail -n 2 $OUT/c2.log | cut -c1-400; exit $rc
