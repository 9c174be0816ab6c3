#!/bin/bash
# round 5, session d: diagnosis after session b's abort -- smoke (environment), then one small matrix-core launch per
# (K, ring) with HIP error logging, each step under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -n 2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
AMD_LOG_LEVEL=1 timeout -k 10 180 python -u -X faulthandler tools/mfma_diag.py > $OUT/diag.log 2>&1; rc=$?; tail -n 30 $OUT/diag.log; exit $rc
