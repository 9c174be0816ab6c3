set -u
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14"
for d in 0 1 2 3; do
  timeout -k 10 300 python -u tools/ab_tiles.py --lines "$L" --modes=-1,1 --env "SPMM_HIP_TILE_DBG=$d" --rounds 3 > gpurun_out/s3/dbg$d.jsonl 2>>gpurun_out/s3/err.log || exit $?
done
D="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14"
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  n=$(echo $pmc | cut -c1-12 | tr ' ' _)
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/s3/pmc_$n -o run -- python3 tools/ab_tiles.py --lines "$D" --modes=1 --rounds 1 --iters 2 > gpurun_out/s3/pmc_$n.log 2>&1 || exit $?
done
echo done
