#!/bin/bash
# round 6, session x: the wide-window POLICY (fp64, K = 32, >= 2.5 M nonzeros, rows averaging >= 256) --
# parity, then the policy against the default window (SPMM_HIP_CAP=2048) on the hold-out avg-100/500 lines (every 80th
# medium-dataset line at offset 40, none in the forced A/B; tools/r06_wide_holdout.txt), K = 32, plan cap recorded
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_widecap.py tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 800 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_wide_holdout.txt)" \
    --k 32 --plans "off:SPMM_HIP_CAP=2048;policy:" --launches 10 --repeat 2 --plan-fields cap \
    > $OUT/wide_holdout.jsonl 2> $OUT/wide_holdout.err
rc=$?; wc -l $OUT/wide_holdout.jsonl; exit $rc
