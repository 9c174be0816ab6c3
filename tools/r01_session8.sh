#!/bin/bash
# Medium-dataset sample sweep (every 160th line, K in {1,8,32,128}) with the column-window policy + generator v2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s8
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run sweep 1100 python tools/sweep.py --dataset medium --stride 160 --k 1,8,32,128 --budget 900 --out $OUT/sweep_medium_s160_v5.jsonl
echo "=== done"
