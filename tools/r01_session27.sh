#!/bin/bash
# Config 3 "rocprof HBM-BW per matrix": PMC traffic (separate rocprofv3 --pmc passes) for representative medium-dataset
# classes at K=32; the bench line of each run gives the kernel time the traffic is divided by.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s27
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for g in "28508159 28508159 5 1.6667 normal random 0.6 1000 0.05 0.05 14" \
         "962627 962627 20 6.6667 normal random 0.3 100 0.95 0.95 14" \
         "445906 445906 100 33.3333 normal random 0.05 0 0.95 0.05 14" \
         "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14" \
         "6158235 6158235 20 6.6667 normal random 0.6 10000 0.05 0.5 14" \
         "65535 65535 5 1.6667 normal random 0.05 0 0.05 0.05 14"; do
    i=$((i+1))
    echo "=== $i $g $(date +%T)"
    timeout -k 10 900 python tools/collect_pmc.py --gen "$g" --k 32 --tag medium_$i --no-latest --steps 10 > $OUT/pmc_$i.log 2>&1
    rc=$?; tail -n 2 $OUT/pmc_$i.log; [ $rc -eq 0 ] || { echo "STOP rc=$rc"; exit $rc; }
    timeout -k 10 300 python bench.py --gen "$g" --k 32 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$i.log 2>&1 || exit 1
    tail -n 1 $OUT/bench_$i.log | cut -c1-200
done
echo "=== done"
