set -u
mkdir -p gpurun_out/s6
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14;1082401 1082401 10 3.3333 normal random 0.6 100 0.95 0.95 14"
for r in 32 64; do for d in 0 1 7; do
  timeout -k 10 300 python -u tools/ab_tiles.py --lines "$L" --modes=-1,1 --env "SPMM_HIP_TILE_DBG=$d;SPMM_HIP_TILE_ROWS=$r" --rounds 3 > gpurun_out/s6/r${r}_dbg$d.jsonl 2>>gpurun_out/s6/err.log || exit $?
done; done
echo done
