#!/bin/bash
# Vector lanes: full GPU suite, then lanes off / policy / forced across densities and K.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s11
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
V1="16,1,1,0,0,0,0,0,0"
V="16,1,0,1,0,0,0,0,0"
S1="$V1,-1;$V1,0;$V1,4;$V1,16;$V1,64"
S="$V,-1;$V,0;$V,2;$V,4;$V,16"
M500="303884 303884 500 166.6667 normal random 0.6 100 1.4 0.95 14"
M500s="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14"
M100="445906 445906 100 33.3333 normal random 0.05 0 0.95 0.05 14"
M50="388875 388875 50 16.6667 normal random 0.3 0 0.5 0.05 14"
run f1 300 python tools/tune_kernel.py --rounds 3 --k 1 --variants "$S1"
run f2 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M500" --variants "$S1"
run f3 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M500" --variants "$S"
run f4 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "$M500" --variants "$S"
run f5 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M500s" --variants "$S1"
run f6 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M500s" --variants "$S"
run f7 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M100" --variants "$S1"
run f8 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M100" --variants "$S"
run f9 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "$M50" --variants "$S1"
run f10 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "$M50" --variants "$S"
run f11 300 python tools/tune_kernel.py --rounds 3 --k 8 --variants "$S"
run f12 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "$M500s" --variants "$S"
echo "=== done"
