set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s21
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s21/prof -o run -- python3 tools/split_probe.py --lines "$(cat tools/split_probe_lines.txt)" --k 32 --settings "default" --rounds 3 --iters 20 > gpurun_out/s21/probe.jsonl 2> gpurun_out/s21/probe.err || { tail -5 gpurun_out/s21/probe.err; exit 1; }
python3 - <<'PY'
import csv, json, collections
rows = list(csv.DictReader(open('gpurun_out/s21/prof/run_kernel_trace.csv')))
# group engine dispatches in order; the probe runs lines sequentially, rounds*(iters+1) launches each
names = collections.Counter(r['Kernel_Name'][:60] for r in rows)
print(names.most_common(8))
eng = [r for r in rows if 'spmm_' in r['Kernel_Name']]
per = 3 * 21
lines = [json.loads(l) for l in open('gpurun_out/s21/probe.jsonl')]
for i, d in enumerate(lines):
    seg = eng[i * per:(i + 1) * per]
    ds = sorted((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in seg)
    gaps = sorted((int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3 for a, b in zip(seg, seg[1:]))
    print(d['gen'][:40], 'event ms %.4f' % d['ms']['default'], 'kernel us median %.1f' % ds[len(ds) // 2], 'gap us median %.1f' % gaps[len(gaps) // 2], 'kinds', len(set(r['Kernel_Name'][:40] for r in seg)))
PY
