set -u
export TMPDIR=/tmp
OUT=gpurun_out/s28
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_tiles.log 2>&1 || { tail -30 $OUT/pytest_tiles.log; exit 1; }
tail -1 $OUT/pytest_tiles.log
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14;22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14"
timeout -k 10 300 python -u tools/ab_tiles.py --modes=-1,0,1 --k 64 --dtype f64,f32 --lines "$L" > $OUT/ab_policy_k64.jsonl 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab_policy_k64.jsonl'):
    d=json.loads(l); print(d['gen'][:48], d['k'], d['dtype'], {m: (d[m]['ms'], d[m]['tiles'], d[m]['speedup']) for m in ['-1','0','1']})
"
bash tools/sweep_resumable.sh 10 200 r02_sweep_medium_s16o10_v11 && bash tools/sweep_resumable.sh 14 500 r02_sweep_medium_s16o14_v11
