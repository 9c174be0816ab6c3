set -u
mkdir -p gpurun_out/s11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s11/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s11/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s11/pytest_gpu.log
