#!/bin/bash
# Column windows (chained mode): GPU parity, then A/B of window sizes vs no windows on matrices of each class.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s5
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run wtests 600 python -m pytest tests/test_gpu_windows.py -x -q
W="16,1,0,1,0,0,0,-1;16,1,0,1,0,0,0,0;16,1,0,1,0,0,0,1048576;16,1,0,1,0,0,0,2097152;16,1,0,1,0,0,0,3145728;16,1,0,1,0,0,0,6291456"
W1="16,1,1,0,0,0,0,-1;16,1,1,0,0,0,0,0;16,1,1,0,0,0,0,1048576;16,1,1,0,0,0,0,2097152;16,1,1,0,0,0,0,3145728;16,1,1,0,0,0,0,6291456"
run b1 300 python tools/tune_kernel.py --rounds 3 --k 1 --variants "$W1"
run b2 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "196651 196651 500 166.6667 normal random 0.3 0 0.95 0.05 14" --variants "$W"
run b3 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14" --variants "$W"
run b4 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "445906 445906 100 33.3333 normal random 0.05 0 0.95 0.05 14" --variants "$W"
run b5 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "12192 12192 100 33.3333 normal random 0.05 0 0.05 0.05 14" --variants "$W"
run b6 300 python tools/tune_kernel.py --rounds 3 --k 8 --gen "196651 196651 500 166.6667 normal random 0.3 0 0.95 0.05 14" --variants "$W"
run b7 300 python tools/tune_kernel.py --rounds 3 --k 32 --gen "362298 362298 100 33.3333 normal random 0.6 0 0.5 0.05 14" --variants "$W"
run b8 300 python tools/tune_kernel.py --rounds 3 --k 32 --variants "$W"
echo "=== done"
