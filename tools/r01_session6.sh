#!/bin/bash
# Column-window sizes on the dense wide-span class (K = 8, 32, 128) + policy check; window GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s6
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run wtests 600 python -m pytest tests/test_gpu_windows.py -x -q
V="16,1,0,1,0,0,0"
W32="$V,-1;$V,0;$V,4194304;$V,6291456;$V,8388608;$V,12582912;$V,16777216;$V,25165824"
W8="$V,-1;$V,0;$V,524288;$V,1048576;$V,1572864;$V,2097152;$V,3145728"
M1="196651 196651 500 166.6667 normal random 0.3 0 0.95 0.05 14"
M2="303884 303884 500 166.6667 normal random 0.6 100 1.4 0.95 14"
M3="89418 89418 500 166.6667 normal random 0.6 100 1.4 0.95 14"
M4="72652 72652 500 166.6667 normal random 0.3 1000 1.9 0.5 14"
M5="250268 250268 500 166.6667 normal random 0.3 10000 0.05 0.5 14"
M6="980644 980644 100 33.3333 normal random 0.3 100 1.4 0.95 14"
run c1 300 python tools/tune_kernel.py --rounds 2 --k 32 --gen "$M1" --variants "$W32"
run c2 300 python tools/tune_kernel.py --rounds 2 --k 8 --gen "$M1" --variants "$W8"
run c3 400 python tools/tune_kernel.py --rounds 2 --k 32 --gen "$M2" --variants "$W32"
run c4 400 python tools/tune_kernel.py --rounds 2 --k 8 --gen "$M2" --variants "$W8"
run c5 300 python tools/tune_kernel.py --rounds 2 --k 32 --gen "$M3" --variants "$W32"
run c6 300 python tools/tune_kernel.py --rounds 2 --k 32 --gen "$M4" --variants "$W32"
run c7 300 python tools/tune_kernel.py --rounds 2 --k 32 --gen "$M5" --variants "$W32"
run c8 300 python tools/tune_kernel.py --rounds 2 --k 128 --gen "$M1" --variants "$W32"
run c9 300 python tools/tune_kernel.py --rounds 2 --k 32 --gen "$M6" --variants "$W32"
run c10 300 python tools/tune_kernel.py --rounds 2 --k 8 --gen "$M3" --variants "$W8"
echo "=== done"
