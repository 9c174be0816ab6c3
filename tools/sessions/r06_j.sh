#!/bin/bash
# round 6, session j: the paired-rows POLICY (reuse-gated) on 60 hold-out avg-5 lines
# (tools/r06_pair_holdout.txt: every 40th dataset line at offset 20, none in the fit), policy against pairing off,
# fp64 K 8 / 32 and fp32 K 32; then the pair parity tests again on this build
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L="$(paste -sd';' tools/r06_pair_holdout.txt)"
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$L" --k 8,32 --plans "off:SPMM_HIP_PAIR=-1;policy:" \
    --launches 10 --repeat 2 > $OUT/holdout_f64.jsonl 2> $OUT/holdout_f64.err || exit $?
wc -l $OUT/holdout_f64.jsonl
timeout -k 10 600 python -u tools/mfma_engine_trace.py --lines "$L" --k 32 --dtype f32 \
    --plans "off:SPMM_HIP_PAIR=-1;policy:" --launches 10 --repeat 2 > $OUT/holdout_f32.jsonl 2> $OUT/holdout_f32.err
rc=$?; wc -l $OUT/holdout_f32.jsonl; exit $rc
