set -u
export TMPDIR=/tmp
OUT=gpurun_out/final2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python tools/collect_pmc.py --tag r02 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-700
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rocprof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload pipeline --steps 200 --warmup 20 > $OUT/pipe512.log 2>&1 || exit 1
tail -1 $OUT/pipe512.log | cut -c1-300
