#!/bin/bash
# v8 inspector (128-B panels for low-similarity rows with 4-12 L2 spans; tiny-row windows gated on row similarity):
# GPU suite, policy-vs-old A/B on the three triggering probe matrices, medium sample at K=1,8,32,128.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s24
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
i=0
for g in "388875 388875 50 16.6667 normal random 0.3 0 0.5 0.05 14" \
         "1787736 1787736 20 6.6667 normal random 0.05 0 0.5 0.05 14" \
         "1515383 1515383 100 33.3333 normal random 0.05 0 0.95 0.05 14"; do
    i=$((i+1))
    for k in 32 128; do
        run ab_${i}_k$k 300 python tools/tune_kernel.py --gen "$g" --k $k --rounds 3 --iters 5 \
            --variants "16,1,0,1,0,0,0;16,1,0,1,0,0,32"
    done
done
run sweep 1200 python tools/sweep.py --stride 160 --k 1,8,32,128 --out $OUT/sweep_s160_v8.jsonl
echo "=== done"
