#!/usr/bin/env python3
"""tools/pmc_class_table.py -- the gather-ceiling table per (avg nonzeros per row, bw) class from tools/pmc_dataset.py
records: per class the matrices, the median and p10/p90 fraction of the gather ceiling
(frac_of_achievable), the median compulsory roofline fraction, the median past-L2 traffic over the algorithmic bytes,
the median L2 hit rate and the ceiling's binding term (past-L2 gather / L2 requests), plus the matrix-core share
(plans with tiles).  Classes under 0.5 of their ceiling are the ones a kernel change can still move.

  python tools/pmc_class_table.py profiles/r04/pmc/pmc_strat_p*.jsonl
"""
import argparse
import glob
import json
from collections import defaultdict

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    args = ap.parse_args()
    recs = {}
    for pat in args.files:
        for f in glob.glob(pat):
            for l in open(f):
                if l.startswith("{"):
                    r = json.loads(l)
                    recs[(r["gen"], r["k"], r["dtype"])] = r
    cls = defaultdict(list)
    for r in recs.values():
        g = r["gen"].split()
        cls[(int(g[2]), float(g[6]))].append(r)
    print(f"{len(recs)} matrices, {len(cls)} classes, engine {sorted({r['engine_sha256'][:8] for r in recs.values()})}\n")
    print("| avg | bw | matrices | frac of ceiling: median (p10–p90) | compulsory frac median | past-L2 / alg bytes | "
          "L2 hit | bound: gather / L2 req | with tiles |")
    print("|---|---|---|---|---|---|---|---|---|")
    allf = []
    for key in sorted(cls):
        rs = cls[key]
        fa = np.array([r["frac_of_achievable"] for r in rs if r.get("frac_of_achievable") is not None])
        allf += list(fa)
        fr = np.median([r["roofline_frac"] for r in rs])
        tr = np.median([r["traffic_over_alg"] for r in rs])
        hit = np.median([r["l2_hit"] for r in rs])
        nb = sum(1 for r in rs if r.get("achievable_bound") == "L2 requests")
        ng = sum(1 for r in rs if r.get("achievable_bound") == "past-L2 gather")
        nt = sum(1 for r in rs if r.get("tiles", 0) > 0)
        print(f"| {key[0]} | {key[1]} | {len(rs)} | {np.median(fa):.2f} ({np.percentile(fa, 10):.2f}–"
              f"{np.percentile(fa, 90):.2f}) | {fr:.3f} | {tr:.2f} | {hit:.2f} | {ng} / {nb} | {nt} |")
    allf = np.array(allf)
    print(f"| **all** | | {len(recs)} | **{np.median(allf):.2f}** ({np.percentile(allf, 10):.2f}–"
          f"{np.percentile(allf, 90):.2f}) | {np.median([r['roofline_frac'] for r in recs.values()]):.3f} | | | | |")


if __name__ == "__main__":
    main()
