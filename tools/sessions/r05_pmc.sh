#!/bin/bash
# round 5 (verdict r04 item 3): per-matrix PMC traffic on the stratified medium-dataset set, 40 lines per (avg, bw)
# class (<= 40 M nonzeros), shipped build, one K per call:  bash tools/sessions/r05_pmc.sh <K>
set -u
cd "${GRAFT_REPO_ROOT:-.}"
K=$1
OUT=gpurun_out/r05pmc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/pmc_dataset.py collect --set stratified --per-class 40 --max-nnz 4e7 --k $K \
    --timeout 330 --tag strat_k$K --out $OUT/pmc_strat_k$K.jsonl > $OUT/pmc_strat_k$K.log 2>&1; rc=$?
tail -n 4 $OUT/pmc_strat_k$K.log; exit $rc
