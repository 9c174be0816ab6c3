#!/bin/bash
# round 4: per-matrix PMC traffic on >= 1,000 stratified medium-dataset lines (56 per (avg, bw) class, <= 40 M
# nonzeros), K=32 fp64, final build; one part of the set per call:  bash tools/sessions/r04_pmc_part.sh <i> <n>
set -u
cd "${GRAFT_REPO_ROOT:-.}"
I=$1; N=$2
OUT=gpurun_out/r04pmc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/pmc_dataset.py collect --set stratified --per-class 56 --max-nnz 4e7 --part $I/$N \
    --timeout 520 --tag strat_p$I --out $OUT/pmc_strat_p$I.jsonl > $OUT/pmc_strat_p$I.log 2>&1; rc=$?
tail -n 4 $OUT/pmc_strat_p$I.log; exit $rc
