#!/usr/bin/env python3
"""tools/summarize_ab.py -- the matrix-core policy on the medium dataset, per class (BASELINE config 3).

Reads tools/sweep.py A/B records (`--base-env SPMM_HIP_MFMA=-1`: the shipped plan and the plan without matrix-core
tiles, timed interleaved in one process) and prints, per K and per (avg nonzeros per row, bw, cross-row similarity)
class: lines, aggregate GFLOP/s of both plans (sum of flops / sum of time) and their ratio, the geometric mean and
the worst line ratio, the lines below 0.9x / 1.0x, the median roofline fraction of the shipped plan, and the parity
flags (exact rows of both plans bit-identical; the oracle check of the shipped plan).  With --census (the plan
census of the same build, tools/plan_census.py) it also reports how many of the changed (line, K) pairs the records
cover.

  python tools/summarize_ab.py profiles/r04/sweep/ab_changed_8w.jsonl.gz --solo profiles/r04/sweep/ab_recheck_solo.jsonl.gz \
      profiles/r04/sweep/ab_solo.jsonl.gz --census profiles/r04/plan_census.jsonl.gz --only-changed

With --solo, records of those files (the same A/B timed by ONE process alone on the GPU) replace the records of the
same (line, K); with --only-changed only the census' changed pairs are tabulated.  The table then says how many of
each class's timings come from solo runs.
"""
import argparse
import glob
import gzip
import json
import math
from collections import defaultdict

import numpy as np


def load(paths):
    recs = {}
    for p in [f for pat in paths for f in sorted(glob.glob(pat))]:
        op = gzip.open if str(p).endswith(".gz") else open
        for line in op(p, "rt"):
            if line.startswith("{"):
                r = json.loads(line)
                if "ms_base" in r:
                    recs[(r["gen"], r["k"], r.get("dtype", "f64"))] = r
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--census", default=None)
    ap.add_argument("--solo", nargs="*", default=[])
    ap.add_argument("--only-changed", action="store_true")
    args = ap.parse_args()
    recs = load(args.files)
    solo = load(args.solo) if args.solo else {}
    for key, r in solo.items():
        r["_solo"] = True
        recs[key] = r
    out = []
    if args.census:
        changed = set()
        op = gzip.open if args.census.endswith(".gz") else open
        for l in op(args.census, "rt"):
            d = json.loads(l)
            if d.get("mode") == "mfma":
                changed.add((d["gen"], d["k"]))
        have = {(g, k) for (g, k, _dt) in recs}
        out.append(f"Census: {len(changed)} (line, K) pairs take matrix-core tiles; A/B records cover "
                   f"{len(changed & have)} of them ({len(have - changed)} records of other pairs); "
                   f"{sum(1 for (g, k, _d), r in recs.items() if r.get('_solo') and (g, k) in changed)} timed solo.\n")
        if args.only_changed:
            recs = {key: r for key, r in recs.items() if (key[0], key[1]) in changed}
    for K in sorted({k for (_, k, _) in recs}):
        rows = defaultdict(list)
        for (g, k, dt), r in recs.items():
            if k == K:
                p = g.split()
                rows[(int(p[2]), float(p[6]), float(p[9]))].append(r)
        out.append(f"\n### K = {K}\n")
        out.append("| avg | bw | crs | lines (solo) | agg GFLOP/s shipped | agg GFLOP/s no-MFMA | agg ratio | geo-mean | "
                   "worst | < 0.9x | < 1.0x | median frac | parity |")
        out.append("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
        tot = [0.0, 0.0, 0.0, []]
        for key in sorted(rows):
            rs = rows[key]
            fl = sum(2.0 * r["nnz"] * K for r in rs)
            t_on = sum(r["ms"] for r in rs) * 1e-3
            t_off = sum(r["ms_base"] for r in rs) * 1e-3
            sp = np.array([r["ms_base"] / r["ms"] for r in rs])
            fr = np.array([r["roofline_frac"] for r in rs])
            par = all(r.get("bitexact_seq_rows", True) and r.get("normwise_ok", True) and r.get("bitexact_vs_base", True)
                      for r in rs)
            tot[0] += fl
            tot[1] += t_on
            tot[2] += t_off
            tot[3] += list(sp)
            ns = sum(1 for r in rs if r.get("_solo"))
            out.append(f"| {key[0]} | {key[1]} | {key[2]} | {len(rs)} ({ns}) | {fl / t_on / 1e9:,.0f} | {fl / t_off / 1e9:,.0f} | "
                       f"{t_off / t_on:.3f} | {math.exp(np.log(sp).mean()):.3f} | {sp.min():.3f} | {(sp < 0.9).sum()} | "
                       f"{(sp < 1.0).sum()} | {np.median(fr):.3f} | {'ok' if par else 'FAIL'} |")
        sp = np.array(tot[3])
        out.append(f"| **all** | | | {len(sp)} | {tot[0] / tot[1] / 1e9:,.0f} | {tot[0] / tot[2] / 1e9:,.0f} | "
                   f"**{tot[2] / tot[1]:.3f}** | {math.exp(np.log(sp).mean()):.3f} | {sp.min():.3f} | {(sp < 0.9).sum()} | "
                   f"{(sp < 1.0).sum()} | | |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
