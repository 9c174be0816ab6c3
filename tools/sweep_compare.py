#!/usr/bin/env python3
"""tools/sweep_compare.py -- two config-3 sweeps, line by line: for every (generator line, K) both sweeps recorded,
the speedup new / old of the kernel time, summarised per K and per (avg nonzeros per row, bw) class -- geomean,
p10, minimum, share of lines slower than 0.95x -- and the median roofline fraction of each sweep on the common lines.

  python tools/sweep_compare.py profiles/r03_sweep_medium.jsonl.gz profiles/r05_sweep_medium.jsonl.gz
"""
import argparse
import gzip
import json
import math
from collections import defaultdict

import numpy as np

AVGS = (5, 10, 20, 50, 100, 500)
BWS = (0.05, 0.3, 0.6)


def load(path):
    op = gzip.open if path.endswith(".gz") else open
    out = {}
    with op(path, "rt") as f:
        for l in f:
            if l.startswith("{"):
                r = json.loads(l)
                if r.get("dtype", "f64") == "f64" and r.get("ms"):
                    out[(r["gen"], int(r["k"]))] = r
    return out


def klass(gen):
    f = gen.split()
    avg = min(AVGS, key=lambda a: abs(math.log(float(f[2]) / a)))
    bw = min(BWS, key=lambda b: abs(float(f[6]) - b))
    return avg, bw


def stats(sp):
    a = np.array(sp)
    return (float(np.exp(np.log(a).mean())), float(np.percentile(a, 10)), float(a.min()), float((a < 0.95).mean()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("old")
    ap.add_argument("new")
    args = ap.parse_args()
    old, new = load(args.old), load(args.new)
    common = sorted(set(old) & set(new))
    eo = {r.get("engine_sha256", "?")[:8] for r in old.values()}
    en = {r.get("engine_sha256", "?")[:8] for r in new.values()}
    print(f"### Line-by-line: {args.new} (engine {', '.join(sorted(en))}) over {args.old} (engine "
          f"{', '.join(sorted(eo))})\n")
    print(f"{len(common)} (line, K) pairs in both.  Speedup = old kernel time / new kernel time (same line, same K, "
          "fp64; each sweep's own launch timing).\n")
    print("| K | pairs | geomean | p10 | min | share < 0.95x | median frac old | median frac new | aggregate old → new "
          "GFLOP/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    byk = defaultdict(list)
    for key in common:
        byk[key[1]].append(key)
    for k in sorted(byk):
        ks = byk[k]
        sp = [old[x]["ms"] / new[x]["ms"] for x in ks]
        g, p10, mn, slow = stats(sp)
        fo = np.median([old[x]["roofline_frac"] for x in ks])
        fn = np.median([new[x]["roofline_frac"] for x in ks])
        fl = sum(2.0 * old[x]["nnz"] * k for x in ks)
        ago = fl / sum(old[x]["ms"] * 1e-3 for x in ks) / 1e9
        agn = fl / sum(new[x]["ms"] * 1e-3 for x in ks) / 1e9
        print(f"| {k} | {len(ks)} | {g:.3f} | {p10:.3f} | {mn:.3f} | {slow:.3f} | {fo:.3f} | {fn:.3f} | "
              f"{ago:,.0f} → {agn:,.0f} |")
    for k in sorted(byk):
        print(f"\n#### K = {k}, per class (geomean speedup / p10 / median frac old → new)\n")
        print("| avg | bw 0.05 | bw 0.3 | bw 0.6 |")
        print("|---|---|---|---|")
        cls = defaultdict(list)
        for x in byk[k]:
            cls[klass(x[0])].append(x)
        for a in AVGS:
            cells = []
            for b in BWS:
                xs = cls.get((a, b), [])
                if not xs:
                    cells.append("—")
                    continue
                g, p10, _, _ = stats([old[x]["ms"] / new[x]["ms"] for x in xs])
                fo = np.median([old[x]["roofline_frac"] for x in xs])
                fn = np.median([new[x]["roofline_frac"] for x in xs])
                cells.append(f"{g:.2f}× / {p10:.2f} / {fo:.3f} → {fn:.3f}")
            print(f"| {a} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
