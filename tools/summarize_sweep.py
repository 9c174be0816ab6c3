#!/usr/bin/env python3
"""tools/summarize_sweep.py -- per-class summary of medium-dataset sweep records (BASELINE config 3).

Reads tools/sweep.py JSON lines (several files; a (generator line, K, dtype) record is counted once, the LAST file
wins), groups them by the dataset's own classes -- average nonzeros per row {5,10,20,50,100,500} x bandwidth
{0.05,0.3,0.6} -- and prints, per K, one markdown row per class:
    matrices, median / p10 / p90 roofline fraction, median GFLOP/s,
    aggregate GFLOP/s (sum of flops / sum of kernel time) and aggregate algorithmic GB/s (sum of bytes / sum of time).
The roofline fraction is the record's algorithmic bytes / kernel time / 8 TB/s.

  python tools/summarize_sweep.py profiles/r01_sweep_medium_s16_v8.jsonl ... > profiles/medium_class_summary.md
"""
import argparse
import json
from collections import defaultdict

import numpy as np


def load(paths):
    recs = {}
    for p in paths:
        for line in open(p):
            line = line.strip()
            if not line:
                continue
            r = json.loads(line)
            recs[(r["gen"], r["k"], r.get("dtype", "f64"))] = r
    return list(recs.values())


def table(recs, k, title):
    rows = defaultdict(list)
    for r in recs:
        if r["k"] != k:
            continue
        g = r["gen"].split()
        rows[(int(g[2]), float(g[6]))].append(r)
    out = [f"#### {title}: K = {k}", "",
           "| avg nnz/row | bw | matrices | median frac | p10 | p90 | median GFLOP/s | aggregate GFLOP/s | aggregate alg. GB/s |",
           "|---|---|---|---|---|---|---|---|---|"]
    allr = []
    for key in sorted(rows):
        rs = rows[key]
        allr += rs
        out.append(row_line(f"{key[0]}", f"{key[1]:g}", rs))
    out.append(row_line("**all**", "", allr))
    return "\n".join(out) + "\n"


def row_line(a, b, rs):
    fr = np.array([r["roofline_frac"] for r in rs])
    gf = np.array([r["gflops"] for r in rs])
    ms = np.array([r["ms"] for r in rs])
    flops = gf * ms * 1e-3 * 1e9                      # GFLOP/s x s = flop
    gbs = np.array([r["gbs_alg"] for r in rs])
    byts = gbs * ms * 1e-3 * 1e9
    t = ms.sum() * 1e-3
    return (f"| {a} | {b} | {len(rs)} | {np.median(fr):.3f} | {np.percentile(fr, 10):.3f} | "
            f"{np.percentile(fr, 90):.3f} | {np.median(gf):,.0f} | {flops.sum() / t / 1e9:,.0f} | "
            f"{byts.sum() / t / 1e9:,.0f} |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--title", default="Medium dataset sample")
    ap.add_argument("--k", default="1,8,32,128")
    args = ap.parse_args()
    recs = load(args.files)
    mats = len({r["gen"] for r in recs})
    bad = [r for r in recs if not (r.get("bitexact_seq_rows", True) and r.get("normwise_ok", True))]
    print(f"### {args.title}\n\n{mats} matrices, {len(recs)} records, parity failures on the sampled rows: {len(bad)}\n")
    for k in (int(x) for x in args.k.split(",")):
        print(table(recs, k, args.title))


if __name__ == "__main__":
    main()
