#!/bin/bash
# round 6, session p: the LDS x window (spmm_rows_kernel XW) -- parity (its own tests plus the row
# kernel's parity and paired-row suites, whose code path it restructured), then forced windows against none on the
# narrow-band lines of the stride-80 sample (bw x rows <= 16,384; tools/r06_xwin_lines.txt) at K = 1 and 8, same process, interleaved rounds, with the plan's xwin recorded
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06p; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_xwin.py tests/test_gpu_parity.py tests/test_gpu_pair.py -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
L="$(paste -sd';' tools/r06_xwin_lines.txt)"
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$L" --k 1,8 \
    --plans "off:SPMM_HIP_XWIN=-1;on:SPMM_HIP_XWIN=1" --launches 10 --repeat 2 --plan-fields xwin \
    > $OUT/xwin_ab.jsonl 2> $OUT/xwin_ab.err
rc=$?; wc -l $OUT/xwin_ab.jsonl; exit $rc
