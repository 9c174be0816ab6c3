#!/bin/bash
# K=1 column windows on wide-span sparse rows: at K=1 a gather uses 8 B of a 128-B line, while continuing a row's
# chain in the next window costs a 16-B C round trip -- force windows of 0.5..8 MB of B on the slowest K=1 records.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s22
mkdir -p $OUT
V="16,1,1,0,0,0,0,-1;16,1,1,0,0,0,0,524288;16,1,1,0,0,0,0,1048576;16,1,1,0,0,0,0,2097152;16,1,1,0,0,0,0,4194304;16,1,1,0,0,0,0,8388608"
i=0
for g in "13418495 13418495 5 1.6667 normal random 0.6 0 0.95 0.05 14" \
         "3670015 3670015 5 1.6667 normal random 0.6 0 0.5 0.05 14" \
         "14713889 14713889 10 3.3333 normal random 0.3 0 0.95 0.05 14" \
         "18448383 18448383 5 1.6667 normal random 0.05 0 0.95 0.05 14" \
         "4838920 4838920 20 6.6667 normal random 0.6 0 0.95 0.05 14" \
         "1375181 1375181 20 6.6667 normal random 0.6 0 0.5 0.05 14" \
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"; do
    i=$((i+1))
    for k in 1 2; do
        echo "=== $i k=$k $g $(date +%T)"
        timeout -k 10 300 python tools/tune_kernel.py --gen "$g" --k $k --rounds 2 --iters 5 --variants "$V" \
            > $OUT/w_${i}_k$k.log 2>&1
        rc=$?; tail -n 1 $OUT/w_${i}_k$k.log | cut -c1-240
        case $rc in 0|1) ;; *) echo "STOP rc=$rc"; exit $rc ;; esac
    done
done
echo "=== done"
