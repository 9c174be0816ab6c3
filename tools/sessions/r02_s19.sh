set -u
mkdir -p gpurun_out/s19
L=spmm-research_amd/lib_ab
export SPMM_HIP_TILES=1
timeout -k 10 600 python -u tools/ab_libs.py --lib $L/w3_u12.so --lib $L/w4_u8.so --lib $L/w2_u20.so \
  --gen "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14" \
  --gen "39120 39120 500 166.6667 normal random 0.05 0 1.4 0.95 14" \
  --gen "22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14" \
  --gen "39120 39120 500 166.6667 normal random 0.3 0 0.5 0.95 14" \
  --k 32 --rounds 5 > gpurun_out/s19/ab_occ.jsonl 2> gpurun_out/s19/ab_occ.err || { tail -20 gpurun_out/s19/ab_occ.err; exit 1; }
cat gpurun_out/s19/ab_occ.jsonl
