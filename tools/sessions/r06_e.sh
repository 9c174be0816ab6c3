#!/bin/bash
# round 6, session e: (1) fused vs separate split-row combine on small skewed lines (K 1 / 8 / 32), the tail the
# small-launch breakdown found; (2) ADVICE r05: the fp32 matrix-core gate on hold-out lines (not in the round-5 fit),
# policy against tiles off, K 32 / 128.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_skew_small_lines.txt)" \
    --k 1,8,32 --plans "pol:;nofuse:SPMM_HIP_FUSE=0" --launches 20 > $OUT/fuse.jsonl 2> $OUT/fuse.err
rc=$?; wc -l $OUT/fuse.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/mfma_engine_trace.py --lines "$(paste -sd';' tools/r06_f32_holdout_sub.txt)" \
    --k 32,128 --dtype f32 --plans "pol:;off:SPMM_HIP_MFMA=-1" --launches 10 --repeat 2 > $OUT/f32.jsonl 2> $OUT/f32.err
rc=$?; wc -l $OUT/f32.jsonl; exit $rc
