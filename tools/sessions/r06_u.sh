#!/bin/bash
# round 6, session u: the shipped engine (08e48ee7) on the metric's sample at the other K of config 3 (1, 8, 128; the
# headline is K = 32): the bench line's dataset record per K, no CPU leg, no config-2 sub-record
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06u; mkdir -p $OUT
export TMPDIR=/tmp
for K in 1 8 128; do
  timeout -k 10 400 python -u bench.py --k $K --steps 10 --warmup 3 --no-cpu-baseline --no-config2 \
      --dataset-out $OUT/ds_k$K.jsonl > $OUT/bench_k$K.json 2> $OUT/bench_k$K.err
  rc=$?; tail -c 200 $OUT/bench_k$K.json; echo; [ $rc -eq 0 ] || exit $rc
done
