set -u
mkdir -p gpurun_out/s23
timeout -k 10 400 python -u tools/split_probe.py --lines "$(cat tools/small_m_lines.txt)" --k 1,8,32,128 --settings "default;SPMM_HIP_SEQ_MAX=64;SPMM_HIP_SEQ_MAX=112" --rounds 3 > gpurun_out/s23/probe.jsonl 2> gpurun_out/s23/probe.err || { tail -5 gpurun_out/s23/probe.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/s23/probe.jsonl'):
    d=json.loads(l); b=d['ms']['default']; print(d['gen'][:48], d['k'], 'T', d['plan']['default']['T'], 'lmax', d['plan']['default']['lmax'], '%.1f us'%(b*1e3), {k[-6:]: round(v/b,2) for k,v in d['ms'].items()})
"
