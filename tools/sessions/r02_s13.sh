set -u
mkdir -p gpurun_out/s13
L=spmm-research_amd/lib_ab
export SPMM_HIP_TILES=1
timeout -k 10 600 python -u tools/ab_libs.py --lib $L/old.so --lib $L/dma_nojoint.so --lib $L/dma_joint.so --lib $L/vgpr_nojoint.so --lib $L/vgpr_joint.so \
  --gen "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14" \
  --gen "22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14" \
  --gen "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14" \
  --gen "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14" \
  --k 32 --rounds 5 > gpurun_out/s13/ab_stage.jsonl 2> gpurun_out/s13/ab_stage.err || { tail -20 gpurun_out/s13/ab_stage.err; exit 1; }
cat gpurun_out/s13/ab_stage.jsonl
