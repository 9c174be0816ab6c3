set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tiles_test.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -25 gpurun_out/tiles_test.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u tools/ab_tiles.py --k 32 --dtype f64 > gpurun_out/ab_tiles_k32.jsonl 2> gpurun_out/ab_tiles.err; rc=$?
echo "ab rc=$rc"; cat gpurun_out/ab_tiles_k32.jsonl | cut -c1-600; tail -5 gpurun_out/ab_tiles.err
