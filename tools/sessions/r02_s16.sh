set -u
mkdir -p gpurun_out/s16b
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s16b/pytest.log 2>&1 || { tail -30 gpurun_out/s16b/pytest.log; exit 1; }
tail -1 gpurun_out/s16b/pytest.log
timeout -k 10 300 python bench.py --workload pipeline --steps 200 --warmup 20 > gpurun_out/s16b/pipe512.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload pipeline --steps 200 --warmup 20 --pipe-m 2048 > gpurun_out/s16b/pipe2048.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s16b/prof_pipe -o run -- python3 bench.py --workload pipeline --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/s16b/pipe_prof.log 2>&1 || exit 1
for f in pipe512 pipe2048; do tail -1 gpurun_out/s16b/$f.log | cut -c1-330; done
