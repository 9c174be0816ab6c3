set -u
mkdir -p gpurun_out/s12
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s12/pytest_tiles.log 2>&1 || { tail -30 gpurun_out/s12/pytest_tiles.log; exit 1; }
tail -2 gpurun_out/s12/pytest_tiles.log
timeout -k 10 600 python -u tools/ab_tiles.py --k 32 --dtype f64 --modes=-1,0,1 > gpurun_out/s12/ab_k32_f64.jsonl 2> gpurun_out/s12/ab_k32_f64.err || exit 1
timeout -k 10 300 python -u tools/ab_tiles.py --k 64 --dtype f32 --modes=-1,1 > gpurun_out/s12/ab_k64_f32.jsonl 2> gpurun_out/s12/ab_k64_f32.err || exit 1
python3 -c "
import json
for f in ['gpurun_out/s12/ab_k32_f64.jsonl','gpurun_out/s12/ab_k64_f32.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['gen'][:40], d['k'], d['dtype'], {m: (d[m]['ms'], d[m].get('speedup')) for m in d if m.lstrip('-').isdigit()})
"
