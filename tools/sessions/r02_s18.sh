set -u
mkdir -p gpurun_out/s18
timeout -k 10 600 python -u tools/split_probe.py --lines "$(cat tools/split_probe_lines.txt)" --k 32,8 > gpurun_out/s18/split_probe.jsonl 2> gpurun_out/s18/split_probe.err || { tail -5 gpurun_out/s18/split_probe.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/s18/split_probe.jsonl'):
    d=json.loads(l); b=d['ms']['default']
    print(d['gen'][:36], d['k'], 'T', d['plan']['default']['T'], {k.replace('SPMM_HIP_',''): round(b/v,2) for k,v in d['ms'].items()}, '%.4f'%b)
"
