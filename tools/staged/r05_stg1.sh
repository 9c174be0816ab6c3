#!/bin/bash
# round 5: staged-rows kernel -- GPU parity (tests/test_gpu_staged.py), then an A/B of whole launches on 24 lines
# (avg 20 / 50 / 100 / 500 x small / medium / large, tools/r05_staged_lines.txt) at K 8 / 32 / 128:
# rows = staged rows off (the round-5 policy before them), stg = staged rows forced (no tiles), pol = the policy.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${STG_TAG:-stg1}   # (run with the integration patch applied); mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_staged.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1
rc=$?; tail -n 5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r05_staged_lines.txt)" \
    --k 8,32,128 --plans "rows:SPMM_HIP_STAGED=-1;stg:SPMM_HIP_STAGED=1,SPMM_HIP_TILES=-1;pol:" --launches 20 \
    > $OUT/ab.jsonl 2> $OUT/ab.err
rc2=$?; wc -l $OUT/ab.jsonl; exit $((rc > rc2 ? rc : rc2))
