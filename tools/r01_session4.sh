#!/bin/bash
# A/B of staging / gather addressing / panel width on the medium-sweep regressions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s4
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
V8="16,1,0,1,0,0,0;16,1,0,0,0,0,0;16,1,1,0,0,0,0;16,1,1,1,0,0,0;8,1,0,0,0,0,0;24,1,0,0,0,0,0;16,0,0,0,0,0,0"
V128="16,1,0,1,0,0,0;16,1,0,0,0,0,0;16,1,1,0,0,0,0;16,1,0,1,0,0,32;16,1,0,1,0,0,64;16,1,0,1,0,0,128;16,1,0,0,0,0,32;16,1,0,0,0,0,64"
run a1 300 python tools/tune_kernel.py --rounds 2 --k 8 --gen "303884 303884 500 166.6667 normal random 0.6 100 1.4 0.95 14" --variants "$V8"
run a2 300 python tools/tune_kernel.py --rounds 2 --k 8 --gen "196651 196651 500 166.6667 normal random 0.3 0 0.95 0.05 14" --variants "$V8"
run a3 300 python tools/tune_kernel.py --rounds 2 --k 128 --gen "143035 143035 500 166.6667 normal random 0.05 100 1.4 0.95 14" --variants "$V128"
run a4 300 python tools/tune_kernel.py --rounds 2 --k 128 --gen "111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14" --variants "$V128"
run a5 300 python tools/tune_kernel.py --rounds 2 --k 128 --gen "55886 55886 500 166.6667 normal random 0.3 0 0.5 0.05 14" --variants "$V128"
run a6 300 python tools/tune_kernel.py --rounds 2 --k 128 --gen "202950 202950 10 3.3333 normal random 0.6 100 0.5 0.95 14" --variants "$V128"
run a7 300 python tools/tune_kernel.py --rounds 2 --k 128 --gen "9521746 9521746 10 3.3333 normal random 0.6 100 1.4 0.95 14" --variants "$V128"
run a8 300 python tools/tune_kernel.py --rounds 2 --k 32 --gen "14713889 14713889 10 3.3333 normal random 0.3 0 0.95 0.05 14" --variants "$V8"
echo "=== done"
