set -u
bash tools/evidence.sh r02b || exit $?
timeout -k 10 300 python bench.py --workload pipeline --steps 200 --warmup 20 > gpurun_out/final/pipe512.log 2>&1 || exit 1
tail -1 gpurun_out/final/pipe512.log | cut -c1-300
