#!/bin/bash
# round 4, session g: experiments beside the shipped engine -- the low-register matrix-core tile kernel and its
# B-operand ring variants (tools/mfma_lr.hpp, through the probe ABI), and the cost of the exact fallback
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14;111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14;222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14"
timeout -k 10 400 python -u tools/mfma_probe.py --lr-lib spmm-research_amd/lib/libmfma_probe_lr.so --no-forced --reuse 2 --k 32 --variants np1r12,np1r6 --lines "$L" > $OUT/probe_lr_k32.log 2>&1; rc=$?; grep -c '^{' $OUT/probe_lr_k32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/mfma_probe.py --lr-lib spmm-research_amd/lib/libmfma_probe_lr.so --no-forced --reuse 2 --k 128 --variants np1r12,np2r12,np2r8,np2r6 --lines "$L" > $OUT/probe_lr_k128.log 2>&1; rc=$?; grep -c '^{' $OUT/probe_lr_k128.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mfma_fallback_time.py --k 32,128 > $OUT/fallback.log 2>&1; rc=$?; grep '^{' $OUT/fallback.log | cut -c1-300; exit $rc
