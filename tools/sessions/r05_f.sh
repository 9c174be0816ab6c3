#!/bin/bash
# round 5, session f (verdict r04 item 5): the matrix-core gate's fp32 fit sample -- A/B of the gate
# forced open (SPMM_HIP_MFMA=2) against no matrix-core tiles, same process, on the round-4 fit lines, K 32 / 128, fp32
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1080 python -u tools/sweep.py --dataset tools/r04_fit_lines.txt --k 32,128 --dtype f32 \
    --env SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NPC=96 --base-env SPMM_HIP_MFMA=-1 --workers 6 --budget 900 --check-rows 64 \
    --no-features --iters 10 --out $OUT/fit_ab_f32.jsonl > $OUT/fit_ab_f32.log 2>&1; rc=$?
tail -n 3 $OUT/fit_ab_f32.log; cat $OUT/fit_ab_f32*.jsonl | wc -l; exit $rc
