#!/bin/bash
# v7 evidence + K-panel width / block-cap experiment: GPU suite, smoke, bench, rocprof kernel-trace summary, PMC
# passes, then narrow K panels (64/128-B B rows) and row-group-sized blocks on the low-reuse medium-dataset classes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s20
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 4 $OUT/$name.log | cut -c1-400; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 50 --warmup 10
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
run pmc 900 python tools/collect_pmc.py --tag r01_v7
# U,NTC,DMA,BUF,SEQ_MAX,CAP,PANEL_K[,WIN_BYTES,XCD,LANES]
P="16,1,0,1,0,0,32;16,1,0,1,0,0,16;16,1,0,1,0,0,8;16,1,0,1,0,0,16,-1,1;16,1,0,1,1024,1600,32;16,1,0,1,1024,1024,32"
for g in "1515383 1515383 100 33.3333 normal random 0.05 0 0.95 0.05 14" \
         "362298 362298 100 33.3333 normal random 0.6 0 0.5 0.05 14" \
         "388875 388875 50 16.6667 normal random 0.3 0 0.5 0.05 14" \
         "4838920 4838920 20 6.6667 normal random 0.6 0 0.95 0.05 14" \
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"; do
    n=$(echo $g | cut -d' ' -f1,3,7 | tr ' ' _)
    run panel_$n 300 python tools/tune_kernel.py --gen "$g" --k 32 --rounds 3 --iters 5 --variants "$P"
done
echo "=== done"
