set -u
export TMPDIR=/tmp
OUT=gpurun_out/s26
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_tiles.log 2>&1 || { tail -30 $OUT/pytest_tiles.log; exit 1; }
tail -1 $OUT/pytest_tiles.log
timeout -k 10 500 python -u tools/ab_tiles.py --modes=-1,1,1w2,1w4 --k 32,128 --dtype f64 > $OUT/ab_wide_f64.jsonl 2> $OUT/ab_wide.err || { tail -5 $OUT/ab_wide.err; exit 1; }
timeout -k 10 200 python -u tools/ab_tiles.py --modes=-1,1,1w2,1w4 --k 32 --dtype f32 --lines "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14;111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14" > $OUT/ab_wide_f32.jsonl 2>> $OUT/ab_wide.err || { tail -5 $OUT/ab_wide.err; exit 1; }
python3 -c "
import json,sys
for f in ['$OUT/ab_wide_f64.jsonl','$OUT/ab_wide_f32.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['gen'][:40], d['k'], d['dtype'], {m: (d[m]['ms'], d[m]['speedup'], d[m]['wide'], d[m]['exact_same']) for m in ['-1','1','1w2','1w4']})
"
bash tools/sweep_resumable.sh 10 500 r02_sweep_medium_s16o10_v11
