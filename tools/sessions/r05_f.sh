#!/bin/bash
# round 5, session f (verdict r04 item 5): the matrix-core gate's fit samples on the round-5 tile
# kernel -- A/B of the gate forced open (SPMM_HIP_MFMA=2) against no matrix-core tiles, same process, on every second
# round-4 fit line (tools/r05_fit_lines.txt), K 32 / 128, fp32 and fp64
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1080 python -u tools/sweep.py --dataset tools/r05_fit_lines.txt --k 32,128 --dtype f32,f64 \
    --env SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NPC=96 --base-env SPMM_HIP_MFMA=-1 --workers 6 --budget 900 --check-rows 64 \
    --no-features --iters 10 --out $OUT/fit_ab.jsonl > $OUT/fit_ab.log 2>&1; rc=$?
tail -n 3 $OUT/fit_ab.log; cat $OUT/fit_ab*.jsonl | wc -l; exit $rc
