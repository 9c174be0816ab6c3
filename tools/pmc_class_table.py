#!/usr/bin/env python3
"""tools/pmc_class_table.py -- the gather-ceiling table per (avg nonzeros per row, bw) class from tools/pmc_dataset.py
records: per class the matrices, the median and p10/p90 fraction of the gather ceiling
(frac_of_achievable), the median compulsory roofline fraction, the median past-L2 traffic over the algorithmic bytes,
the median L2 hit rate and the ceiling's binding term (past-L2 gather / L2 requests), plus the matrix-core share
(plans with tiles).  Classes under 0.5 of their ceiling are the ones a kernel change can still move.

  python tools/pmc_class_table.py profiles/r04/pmc/pmc_strat_p*.jsonl
  python tools/pmc_class_table.py --recompute profiles/r05/pmc/pmc_strat_k1.jsonl

--recompute re-derives every record's ceiling with bench.achievable as it stands (round 6: plus the HBM term, the
compulsory bytes at 8 TB/s -- the gather terms alone priced A's streamed bytes at an on-chip rate) and prints the
recorded (gather-only) median beside it.
"""
import argparse
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--recompute", action="store_true", help="re-derive the ceiling with bench.achievable (HBM term)")
    args = ap.parse_args()
    recs = {}
    for pat in args.files:
        for f in glob.glob(pat):
            for l in open(f):
                if l.startswith("{"):
                    r = json.loads(l)
                    recs[(r["gen"], r["k"], r["dtype"])] = r
    if args.recompute:
        import bench
        for r in recs.values():
            r["frac_of_achievable_r05"] = r.get("frac_of_achievable")
            s_ = 8 if r["dtype"] == "f64" else 4
            a = bench.achievable(r["kernel_ms"], r["traffic_bytes"], r.get("tcc_req"), float(r["ncols"]) * r["k"] * s_,
                                 r["bytes_alg"])
            r["frac_of_achievable"] = a["frac_of_achievable"]
            r["achievable_bound"] = a["bound"]
    cls = defaultdict(list)
    for r in recs.values():
        g = r["gen"].split()
        cls[(int(g[2]), float(g[6]))].append(r)
    print(f"{len(recs)} matrices, {len(cls)} classes, engine {sorted({r['engine_sha256'][:8] for r in recs.values()})}\n")
    rc = args.recompute
    print("| avg | bw | matrices | frac of ceiling: median (p10–p90) | " + ("gather-only ceiling (r05) median | " if rc
                                                                          else "")
          + "compulsory frac median | past-L2 / alg bytes | L2 hit | bound: gather / L2 req / HBM | with tiles |")
    print("|---|---|---|---|---|---|---|---|---|" + ("---|" if rc else ""))
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
        nh = sum(1 for r in rs if r.get("achievable_bound") == "HBM compulsory")
        old_ = (f"{np.median([r['frac_of_achievable_r05'] for r in rs]):.2f} | " if rc else "")
        print(f"| {key[0]} | {key[1]} | {len(rs)} | {np.median(fa):.2f} ({np.percentile(fa, 10):.2f}–"
              f"{np.percentile(fa, 90):.2f}) | {old_}{fr:.3f} | {tr:.2f} | {hit:.2f} | {ng} / {nb} / {nh} | {nt} |")
    allf = np.array(allf)
    old_all = (f"{np.median([r['frac_of_achievable_r05'] for r in recs.values()]):.2f} | " if rc else "")
    print(f"| **all** | | {len(recs)} | **{np.median(allf):.2f}** ({np.percentile(allf, 10):.2f}–"
          f"{np.percentile(allf, 90):.2f}) | {old_all}{np.median([r['roofline_frac'] for r in recs.values()]):.3f} | | | | |")


if __name__ == "__main__":
    main()
