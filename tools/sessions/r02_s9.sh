set -u
mkdir -p gpurun_out/s9
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s9/pipe_test.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -30 gpurun_out/s9/pipe_test.log
