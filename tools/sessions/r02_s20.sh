set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 900 python tools/collect_pmc.py --tag r02 > gpurun_out/final/pmc.log 2>&1 || { tail -20 gpurun_out/final/pmc.log; exit 1; }
tail -5 gpurun_out/final/pmc.log
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/final/bench.log 2>&1 || { tail -5 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log
