#!/bin/bash
# Streamed long rows: policy/parity tests, then staged vs streamed A/B on long-row medium-dataset matrices.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s28
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_policies 600 python -u -m pytest tests/test_gpu_policies.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" $OUT/pytest_policies.log && ! grep -q "failed" $OUT/pytest_policies.log || { echo "STOP: policy tests"; exit 1; }
V="16,1,0,1,0,0,0,0,0,0,-1;16,1,0,1,0,0,0,0,0,0,1"
i=0
for g in "39120 39120 500 166.6667 normal random 0.05 0 0.95 0.95 14" \
         "55886 55886 500 166.6667 normal random 0.3 0 0.5 0.05 14" \
         "143035 143035 500 166.6667 normal random 0.05 0 1.4 0.95 14" \
         "303884 303884 500 166.6667 normal random 0.6 0 1.4 0.95 14" \
         "22354 22354 500 166.6667 normal random 0.6 0 0.95 0.95 14" \
         "1571 1571 500 166.6667 normal random 0.3 0 1.9 0.5 14" \
         "980644 980644 100 33.3333 normal random 0.3 0 1.4 0.95 14" \
         "445906 445906 100 33.3333 normal random 0.05 0 0.95 0.05 14" \
         "888859 888859 50 16.6667 normal random 0.05 0 1.4 0.95 14"; do
    i=$((i+1))
    for k in 8 32 128; do
        run s_${i}_k$k 300 python tools/tune_kernel.py --gen "$g" --k $k --rounds 3 --iters 5 --variants "$V"
    done
done
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo "=== done"
