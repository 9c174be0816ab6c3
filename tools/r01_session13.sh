#!/bin/bash
# BASELINE config 5: the 52 validation twins, fp64 + fp32, K=32, reference CPU kernel timed in the same run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s14
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run twins 1100 python tools/sweep.py --dataset twins --k 32 --dtype f64,f32 --cpu-baseline 1.5 --budget 950 --out $OUT/twins_k32.jsonl
echo "=== done"
