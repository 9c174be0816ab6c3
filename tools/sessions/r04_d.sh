#!/bin/bash
# round 4, session d: small-matrix one-launch panels -- tests and A/B (off / 16 / 8 columns) on every 8th small line
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_policies.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$(paste -sd';' tools/r04_small_lines.txt)
timeout -k 10 600 python -u tools/mfma_ab.py --lines "$L" --k 32,128 --modes "off:SPMM_HIP_SMALL_KW=0;kw16:SPMM_HIP_SMALL_KW=16;kw8:SPMM_HIP_SMALL_KW=8" --budget 480 > $OUT/ab_small.jsonl 2> $OUT/ab_small.err; rc=$?; wc -l $OUT/ab_small.jsonl; exit $rc
