#!/usr/bin/env python3
"""tools/summarize_sweep.py -- per-class summary of medium-dataset sweep records (BASELINE config 3).

Reads tools/sweep.py JSON lines (several files; a (generator line, K, dtype) record is counted once, the LAST file
wins), groups them by the dataset's own classes -- average nonzeros per row {5,10,20,50,100,500} x bandwidth
{0.05,0.3,0.6} -- and prints, per K, one markdown row per class:
    matrices, median / p10 / p90 roofline fraction, median GFLOP/s,
    aggregate GFLOP/s (sum of flops / sum of kernel time) and aggregate algorithmic GB/s (sum of bytes / sum of time).
The roofline fraction is the record's algorithmic bytes / kernel time / 8 TB/s.

With --pmc (tools/pmc_dataset.py records, K=32), a second table per class: the matrices with per-launch PMC traffic,
their median past-L2 traffic / algorithmic bytes, and the median fraction of the gather ceiling
(bench.achievable: past-L2 bytes at the measured random-row gather rate for B's size, L2 requests at the
L2-resident rate), ranked by the gap to that ceiling.  --engine keeps one engine build's records
(a sha256 prefix; default: every record, with the builds listed).

  python tools/summarize_sweep.py profiles/r03_sweep_medium.jsonl.gz --pmc profiles/r03_pmc_medium_k32.jsonl > ...
"""
import argparse
import gzip
import json
from collections import Counter, defaultdict

import numpy as np


def load(paths, engine=None):
    recs = {}
    for p in paths:
        op = gzip.open if str(p).endswith(".gz") else open
        for line in op(p, "rt"):
            line = line.strip()
            if not line:
                continue
            r = json.loads(line)
            if engine and not r.get("engine_sha256", "").startswith(engine):
                continue
            recs[(r["gen"], r["k"], r.get("dtype", "f64"))] = r
    return list(recs.values())


def achievable_table(pmc_path, engine=None):
    """Per class: PMC matrices, median traffic / alg. bytes, median and p10 fraction of the gather ceiling; ranked."""
    rows = defaultdict(list)
    for line in open(pmc_path):
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        if engine and not r.get("engine_sha256", "").startswith(engine):
            continue
        if r.get("frac_of_achievable") is None:
            continue
        g = r["gen"].split()
        rows[(int(g[2]), float(g[6]))].append(r)
    if not rows:
        return ""
    lines = []
    for key, rs in rows.items():
        fa = np.array([r["frac_of_achievable"] for r in rs])
        lines.append((float(np.median(fa)), key, rs, fa))
    lines.sort(key=lambda x: x[0])
    out = ["#### Gather ceiling, K = 32 (per-matrix PMC; ranked by the gap: lowest fraction of the ceiling first)", "",
           "| avg nnz/row | bw | PMC matrices | median frac | median traffic / alg. bytes | median L2 hit | "
           "median frac of ceiling | p10 | bound (most matrices) |",
           "|---|---|---|---|---|---|---|---|---|"]
    for med, key, rs, fa in lines:
        fr = np.median([r["roofline_frac"] for r in rs])
        to = np.median([r["traffic_over_alg"] for r in rs])
        l2 = np.median([r["l2_hit"] for r in rs])
        bound = Counter(r.get("achievable_bound") for r in rs).most_common(1)[0][0]
        out.append(f"| {key[0]} | {key[1]:g} | {len(rs)} | {fr:.3f} | {to:.2f} | {l2:.2f} | {med:.3f} | "
                   f"{np.percentile(fa, 10):.3f} | {bound} |")
    allfa = np.concatenate([x[3] for x in lines])
    out.append(f"| **all** | | {len(allfa)} | | | | {np.median(allfa):.3f} | {np.percentile(allfa, 10):.3f} | |")
    return "\n".join(out) + "\n"


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


def size_table(recs, k, title):
    """Per nnz bin at one K: the launch-latency-bound small matrices next to the bandwidth-bound large ones."""
    bins = [(0, 1e6, "< 1 M"), (1e6, 4e6, "1-4 M"), (4e6, 16e6, "4-16 M"), (16e6, 64e6, "16-64 M"),
            (64e6, 1e12, ">= 64 M")]
    out = [f"#### {title}: K = {k} by matrix size", "",
           "| nonzeros | | matrices | median frac | p10 | p90 | median GFLOP/s | aggregate GFLOP/s | aggregate alg. GB/s |",
           "|---|---|---|---|---|---|---|---|---|"]
    for lo, hi, name in bins:
        rs = [r for r in recs if r["k"] == k and lo <= r["nnz"] < hi]
        if rs:
            out.append(row_line(name, "", rs))
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
    ap.add_argument("--pmc", default=None, help="tools/pmc_dataset.py records (K=32) for the gather-ceiling table")
    ap.add_argument("--engine", default=None, help="keep records of this engine build only (sha256 prefix)")
    args = ap.parse_args()
    recs = load(args.files, args.engine)
    mats = len({r["gen"] for r in recs})
    bad = [r for r in recs if not (r.get("bitexact_seq_rows", True) and r.get("normwise_ok", True))]
    shas = Counter(r.get("engine_sha256", "untagged")[:12] for r in recs)
    print(f"### {args.title}\n\n{mats} matrices, {len(recs)} records, parity failures on the sampled rows: {len(bad)}; "
          f"engine builds: " + ", ".join(f"{k} ({v} records)" for k, v in shas.most_common()) + "\n")
    for k in (int(x) for x in args.k.split(",")):
        print(table(recs, k, args.title))
    for k in (int(x) for x in args.k.split(",")):
        print(size_table(recs, k, args.title))
    if args.pmc:
        print(achievable_table(args.pmc, args.engine))


if __name__ == "__main__":
    main()
