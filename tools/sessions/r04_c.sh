#!/bin/bash
# round 4, session c: matrix-core gate fit sample -- A/B (gate forced open vs no matrix-core tiles, same process)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1080 python -u tools/sweep.py --dataset tools/r04_fit_lines.txt --k 32,128 --env SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NPC=96 \
    --base-env SPMM_HIP_MFMA=-1 --workers 6 --budget 900 --check-rows 64 --no-features --iters 10 \
    --out $OUT/fit_ab.jsonl > $OUT/fit_ab.log 2>&1; rc=$?; tail -n 3 $OUT/fit_ab.log; cat $OUT/fit_ab*.jsonl | wc -l; exit $rc
