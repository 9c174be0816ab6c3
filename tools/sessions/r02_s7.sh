set -u
mkdir -p gpurun_out/s7
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14;1082401 1082401 10 3.3333 normal random 0.6 100 0.95 0.95 14"
for d in 0; do
timeout -k 10 300 python -u tools/tile_stamps.py --lines "$L" --env "SPMM_HIP_TILE_ROWS=32;SPMM_HIP_TILE_DBG=$d" > gpurun_out/s7/stamps_d$d.jsonl 2>>gpurun_out/s7/err.log || exit $?
done
echo done
