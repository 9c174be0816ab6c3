set -u
mkdir -p gpurun_out/s4
for r in 64 32 16; do
  timeout -k 10 600 python -u tools/ab_tiles.py --modes=-1,1 --env "SPMM_HIP_TILE_ROWS=$r" --rounds 3 > gpurun_out/s4/rows$r.jsonl 2>>gpurun_out/s4/err.log || exit $?
done
echo done
