#!/bin/bash
# Merged row tuples, branch-free FMA phase: policy tests, then tuple size A/B on similar-row matrices without split rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s26
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
V="16,1,0,1,0,0,0,0,0,0,-1;16,1,0,1,0,0,0,0,0,0,2;16,1,0,1,0,0,0,0,0,0,4"
i=0
for g in "12117817 12117817 10 3.3333 normal random 0.05 100 1.4 0.95 14" \
         "28508159 28508159 5 1.6667 normal random 0.3 100 1.4 0.95 14" \
         "980644 980644 100 33.3333 normal random 0.3 0 1.4 0.95 14" \
         "3519605 3519605 20 6.6667 normal random 0.3 0 1.4 0.95 14" \
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"; do
    i=$((i+1))
    for k in 8 32; do
        run m_${i}_k$k 300 python tools/tune_kernel.py --gen "$g" --k $k --rounds 3 --iters 5 --variants "$V"
    done
done
echo "=== done"
