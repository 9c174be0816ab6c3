#!/bin/bash
# Streamed-row kernel: parity, then staged vs streamed (+ XCD policy check) across densities and K.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s10
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run wtests 600 python -m pytest tests/test_gpu_windows.py -x -q
V1="16,1,1,0,0,0,0,0,0"; V1s="8,1,1,0,0,0,0,0,0"
V="16,1,0,1,0,0,0,0,0"; Vs="8,1,0,1,0,0,0,0,0"
S1="$V1,-1;$V1,1;$Vs,1;$V1,0"
S="$V,-1;$V,1;$Vs,1;$V,0"
M500="303884 303884 500 166.6667 normal random 0.6 100 1.4 0.95 14"
M500s="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14"
M100="445906 445906 100 33.3333 normal random 0.05 0 0.95 0.05 14"
M50="388875 388875 50 16.6667 normal random 0.3 0 0.5 0.05 14"
run e1 300 python tools/tune_kernel.py --rounds 3 --k 1 --variants "$S1"
run e2 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M500" --variants "$S1"
run e3 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M500" --variants "$S"
run e4 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "$M500" --variants "$S"
run e5 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M500s" --variants "$S1"
run e6 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M500s" --variants "$S"
run e7 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M100" --variants "$S1"
run e8 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M100" --variants "$S"
run e9 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M50" --variants "$S1"
run e10 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M50" --variants "$S"
run e11 300 python tools/tune_kernel.py --rounds 3 --k 8 --variants "$S"
run e12 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "$M100" --variants "$S"
echo "=== done"
