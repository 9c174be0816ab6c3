set -u
export TMPDIR=/tmp
OUT=gpurun_out/s25
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/sweep_resumable.sh 10 800 r02_sweep_medium_s16o10_v11
