#!/bin/bash
# round 5, session c (verdict r04 item 6): small launches -- the row-block capacity below the policy's on the 270
# small lines (every 8th medium-dataset line under 1 M nonzeros), K = 32, each against the policy plan in the same
# process (interleaved, exact rows compared bit for bit)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05c; mkdir -p $OUT
export TMPDIR=/tmp
for CAP in 256 128; do
  timeout -k 10 600 python -u tools/sweep.py --dataset tools/r04_small_lines.txt --k 32 --env SPMM_HIP_CAP=$CAP --base-env "" \
      --workers 4 --batches 3 --check-rows 64 --no-features --iters 20 --out $OUT/cap$CAP.jsonl > $OUT/cap$CAP.log 2>&1
  rc=$?; tail -n 2 $OUT/cap$CAP.log; cat $OUT/cap$CAP*.jsonl | wc -l; [ $rc -eq 0 ] || exit $rc
done
