#!/usr/bin/env python3
"""Print the variant table of tools/tune_kernel.py logs: window bytes, median ms, windows, segments, nnz/segment."""
import json
import sys

for f in sys.argv[1:]:
    rows, head = [], None
    for line in open(f):
        if line.startswith('{"variant'):
            rows.append(json.loads(line))
        elif line.startswith('{"best'):
            head = json.loads(line)
    if not rows:
        continue
    print(f"== {f}: {head['matrix'] if head else ''} K={head['k'] if head else ''} nnz={head['nnz'] if head else ''}")
    base = rows[0]["median_ms"]
    for r in rows:
        v, p = r["variant"], r["plan"]
        segs = max(p.get("segments", 1), 1)
        print(f"  U={v['U']:>2} win={v.get('WIN_BYTES', 0):>9} xcd={v.get('XCD', 0):>2} lanes={v.get('LANES', 0):>2}"
              f" -> L{p.get('lmax', '-')}/x{p.get('xcd', '-')} exact={p.get('exact_rows', '-')} T={v['SEQ_MAX']:>4}"
              f" {r['median_ms']:8.4f} ms  x{base / r['median_ms']:5.2f}"
              f"  windows={p.get('windows', 1):>4} segs={segs:>9} nnz/seg={(head['nnz'] if head else 0) / segs:7.1f}"
              f"  close={r['close']}")
