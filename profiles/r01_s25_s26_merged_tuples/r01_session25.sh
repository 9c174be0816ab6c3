#!/bin/bash
# Merged row tuples: parity first, then tuple size A/B (off / 2 / 4) on similar-row (crs 0.95) and crs 0.5 matrices.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s25
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_policies 600 python -u -m pytest tests/test_gpu_policies.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" $OUT/pytest_policies.log && ! grep -q "failed" $OUT/pytest_policies.log || { echo "STOP: policy tests"; exit 1; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
V="16,1,0,1,0,0,0,0,0,0,-1;16,1,0,1,0,0,0,0,0,0,2;16,1,0,1,0,0,0,0,0,0,4"
i=0
for g in "980644 980644 100 33.3333 normal random 0.3 100 1.4 0.95 14" \
         "278691 278691 100 33.3333 normal random 0.3 100 0.95 0.95 14" \
         "722198 722198 50 16.6667 normal random 0.6 100 0.95 0.95 14" \
         "3519605 3519605 20 6.6667 normal random 0.3 100 1.4 0.95 14" \
         "12117817 12117817 10 3.3333 normal random 0.05 100 1.4 0.95 14" \
         "28508159 28508159 5 1.6667 normal random 0.3 100 1.4 0.95 14" \
         "143035 143035 500 166.6667 normal random 0.05 100 1.4 0.95 14" \
         "555536 555536 50 16.6667 normal random 0.3 1000 1.9 0.5 14" \
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"; do
    i=$((i+1))
    for k in 8 32 128; do
        run m_${i}_k$k 300 python tools/tune_kernel.py --gen "$g" --k $k --rounds 3 --iters 5 --variants "$V"
    done
done
echo "=== done"
