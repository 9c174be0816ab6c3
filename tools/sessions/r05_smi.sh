#!/bin/bash
# round 5: does the sweep's slow-timing contamination follow the GPU's clocks, power or temperature?  rocm-smi samples
# every 5 s (a bounded loop) beside a 300-s, 8-worker sweep of every 40th medium line at K 1/8/32/128; records carry
# the wall clock of their timed region (t_wall)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/smi; mkdir -p $OUT
export TMPDIR=/tmp OMP_NUM_THREADS=2
( for i in $(seq 1 100); do echo "=== $(date +%s.%N)"; rocm-smi --showclocks --showtemp --showpower --showuse --showmemuse 2>&1; sleep 5; done ) > $OUT/smi.log 2>&1 &
SMI=$!
timeout -k 10 420 python -u tools/sweep.py --stride 40 --offset 7 --k 1,8,32,128 --budget 300 --workers 8 \
    --no-features --check-rows 8 --gold-rows 4 --iters 10 --out $OUT/sw.jsonl > $OUT/sw.log 2>&1
rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
tail -n 2 $OUT/sw.log; cat $OUT/sw.*.jsonl | wc -l; exit $rc
