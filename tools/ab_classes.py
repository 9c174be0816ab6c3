#!/usr/bin/env python3
"""tools/ab_classes.py -- per-class summary of a two-plan A/B from tools/mfma_engine_trace.py.

Per (line, K): the best of each plan's timed rounds; speed-up = base ms / new ms.  Groups by the line's average row
length (generator parameter 3) and a size split at --big nonzeros-equivalent rows x avg; prints per (K, class) the
count, geometric mean, min, max and the time-weighted speed-up (sum of base ms / sum of new ms).

  python tools/ab_classes.py gpurun_out/r06n/ring_ab.jsonl --base off --new on
"""
import argparse
import collections
import json
import math


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jsonl")
    ap.add_argument("--base", default="off")
    ap.add_argument("--new", default="on")
    ap.add_argument("--big", type=float, default=4e6, help="nonzeros (rows x avg) splitting small from big lines")
    ap.add_argument("--json", action="store_true", help="one JSON object per class instead of a table")
    args = ap.parse_args()
    best = collections.defaultdict(dict)
    for ln in open(args.jsonl):
        r = json.loads(ln)
        key = (r["gen"], r["k"])
        ms = r["ms"]
        d = best[key]
        d[r["plan"]] = min(ms, d.get(r["plan"], math.inf))
    cls = collections.defaultdict(list)
    for (gen, k), d in best.items():
        if args.base not in d or args.new not in d:
            continue
        g = gen.split()
        avg = float(g[2])
        size = "big" if float(g[0]) * avg >= args.big else "small"
        cls[(k, avg, size)].append((d[args.base], d[args.new]))
        cls[(k, "all", "all")].append((d[args.base], d[args.new]))
    rows = []
    for key in sorted(cls, key=lambda x: (x[0], str(x[1]), x[2])):
        v = cls[key]
        sp = [a / b for a, b in v]
        gm = math.exp(sum(math.log(x) for x in sp) / len(sp))
        tw = sum(a for a, _ in v) / sum(b for _, b in v)
        rows.append({"k": key[0], "avg": key[1], "size": key[2], "n": len(v), "geomean": round(gm, 3),
                     "min": round(min(sp), 3), "max": round(max(sp), 3), "time_weighted": round(tw, 3),
                     "base_ms": round(sum(a for a, _ in v), 4), "new_ms": round(sum(b for _, b in v), 4)})
    if args.json:
        for r in rows:
            print(json.dumps(r))
        return
    print(f"| K | avg | size | lines | geomean {args.new}/{args.base} speed-up | min | max | time-weighted | ms {args.base} -> {args.new} |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['k']} | {r['avg']} | {r['size']} | {r['n']} | {r['geomean']:.3f} | {r['min']:.3f} | {r['max']:.3f} | "
              f"{r['time_weighted']:.3f} | {r['base_ms']:.3f} -> {r['new_ms']:.3f} |")


if __name__ == "__main__":
    main()
