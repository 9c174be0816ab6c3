set -u
export TMPDIR=/tmp
OUT=gpurun_out/s27
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_tiles.py --modes=-1,0,1 --k 64,128 --dtype f64 --lines "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14;22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14" > $OUT/ab_policy_k128.jsonl 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab_policy_k128.jsonl'):
    d=json.loads(l); print(d['gen'][:48], d['k'], {m: (d[m]['ms'], d[m]['tiles'], d[m]['speedup']) for m in ['-1','0','1']})
"
bash tools/sweep_resumable.sh 10 300 r02_sweep_medium_s16o10_v11 && bash tools/sweep_resumable.sh 14 600 r02_sweep_medium_s16o14_v11
