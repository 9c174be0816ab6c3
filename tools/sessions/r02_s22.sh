set -u
mkdir -p gpurun_out/s22
L="65535 65535 5 1.6667 normal random 0.3 0 0.05 0.5 14;65535 65535 5 1.6667 normal random 0.3 1000 0.05 0.5 14;33825 33825 10 3.3333 normal random 0.3 0 0.05 0.5 14;3483 3483 100 33.3333 normal random 0.3 0 0.05 0.5 14;698 698 500 166.6667 normal random 0.3 0 0.05 0.5 14;2097151 2097151 5 1.6667 normal random 0.3 0 0.05 0.5 14"
timeout -k 10 300 python -u tools/split_probe.py --lines "$L" --k 1,8,32 --settings "default;SPMM_HIP_SEQ_MAX=64;SPMM_HIP_SEQ_MAX=2048" > gpurun_out/s22/probe.jsonl 2> gpurun_out/s22/probe.err || { tail -5 gpurun_out/s22/probe.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/s22/probe.jsonl'):
    d=json.loads(l); print(d['gen'][:44], d['k'], 'nnz', d['nnz'], {k[-8:]: round(v*1e3,1) for k,v in d['ms'].items()}, 'T', d['plan']['default']['T'], 'blocks', d['plan']['default']['blocks'])
"
