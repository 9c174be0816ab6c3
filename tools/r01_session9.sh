#!/bin/bash
# XCD-contiguous block order: parity, then on/off A/B (config 2 at K=1/8/32, narrow-band K=1/8 matrices).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s9
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run wtests 600 python -m pytest tests/test_gpu_windows.py -x -q
V1="16,1,1,0,0,0,0"
V="16,1,0,1,0,0,0"
X1="$V1,-1,-1;$V1,-1,1;$V1,0,0"
X="$V,-1,-1;$V,-1,1;$V,0,0"
run d1 300 python tools/tune_kernel.py --rounds 3 --k 1 --variants "$X1"
run d2 300 python tools/tune_kernel.py --rounds 3 --k 8 --variants "$X"
run d3 300 python tools/tune_kernel.py --rounds 3 --k 32 --variants "$X"
run d4 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "1600000 1600000 20 6.6667 normal random 0.05 100 0.95 0.5 14" --variants "$X1"
run d5 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "1600000 1600000 20 6.6667 normal random 0.05 100 0.95 0.5 14" --variants "$X"
run d6 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "5242879 5242879 5 1.6667 normal random 0.05 0 0.5 0.05 14" --variants "$X1"
run d7 300 python tools/tune_kernel.py --rounds 3 --k 1 --gen "2097151 2097151 5 1.6667 normal random 0.3 100 0.95 0.95 14" --variants "$X1"
run d8 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "400000 400000 20 6.6667 normal random 0.01 100 0.95 0.5 14" --variants "$X"
echo "=== done"
