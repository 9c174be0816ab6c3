set -u
mkdir -p gpurun_out/s8
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s8/tiles_test.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s8/tiles_test.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/r02_s7.sh || exit $?
for r in 32 64; do
  timeout -k 10 600 python -u tools/ab_tiles.py --modes=-1,1 --env "SPMM_HIP_TILE_ROWS=$r" --rounds 3 > gpurun_out/s8/rows$r.jsonl 2>>gpurun_out/s8/err.log || exit $?
done
echo done
