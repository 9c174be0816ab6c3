#!/bin/bash
# Tiny-row (K=1/2) window policy + DLMC input: GPU suite, policy-vs-off A/B on the K=1 probe matrices, K=1/2 medium sample.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s23
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
i=0
for g in "13418495 13418495 5 1.6667 normal random 0.6 0 0.95 0.05 14" \
         "3670015 3670015 5 1.6667 normal random 0.6 0 0.5 0.05 14" \
         "4838920 4838920 20 6.6667 normal random 0.6 0 0.95 0.05 14" \
         "1375181 1375181 20 6.6667 normal random 0.6 0 0.5 0.05 14" \
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"; do
    i=$((i+1))
    for k in 1 2; do
        run ab_${i}_k$k 300 python tools/tune_kernel.py --gen "$g" --k $k --rounds 3 --iters 5 \
            --variants "16,1,1,0,0,0,0,0;16,1,1,0,0,0,0,-1"
    done
done
run sweep_k12 900 python tools/sweep.py --stride 160 --k 1,2 --out $OUT/sweep_s160_k12_v8.jsonl
echo "=== done"
