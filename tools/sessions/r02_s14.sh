set -u
mkdir -p gpurun_out/s14
L=spmm-research_amd/lib_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s14/pytest_tiles.log 2>&1 || { tail -30 gpurun_out/s14/pytest_tiles.log; exit 1; }
tail -1 gpurun_out/s14/pytest_tiles.log
SPMM_HIP_TILES=1 timeout -k 10 600 python -u tools/ab_libs.py --lib $L/nodpp.so --lib $L/dpp.so \
  --gen "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14" \
  --gen "22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14" \
  --gen "22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14" \
  --gen "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14" \
  --gen "222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14" \
  --k 32,128 --rounds 5 > gpurun_out/s14/ab_dpp.jsonl 2> gpurun_out/s14/ab_dpp.err || { tail -20 gpurun_out/s14/ab_dpp.err; exit 1; }
cat gpurun_out/s14/ab_dpp.jsonl
timeout -k 10 600 python -u tools/ab_tiles.py --k 32 --dtype f64 --modes=-1,1 --rounds 3 > gpurun_out/s14/ab_tiles_k32.jsonl 2> gpurun_out/s14/ab_tiles_k32.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s14/ab_tiles_k32.jsonl'):
    d=json.loads(l); print(d['gen'][:44], {m: (d[m]['ms'], d[m].get('speedup'), d[m].get('frac')) for m in d if m.lstrip('-').isdigit()})
"
