#!/bin/bash
# K-panel width probe: 256-B vs 128-B B-row panels (kw 32 vs 16 fp64) on the 41 medium-sample matrices with
# >= 20 nnz/row and >= 5 M nnz, at K=32 and K=128 (one tune_kernel process per matrix and K).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s21
mkdir -p $OUT
i=0
while read -r g; do
    i=$((i+1))
    for k in 32 128; do
        echo "=== $i k=$k $g $(date +%T)"
        timeout -k 10 240 python tools/tune_kernel.py --gen "$g" --k $k --rounds 2 --iters 5 \
            --variants "16,1,0,1,0,0,32;16,1,0,1,0,0,16" > $OUT/p_${i}_k$k.log 2>&1
        rc=$?; tail -n 1 $OUT/p_${i}_k$k.log | cut -c1-200
        case $rc in 0|1) ;; *) echo "STOP rc=$rc"; exit $rc ;; esac
    done
done < tools/panel_probe_lines.txt
echo "=== done"
