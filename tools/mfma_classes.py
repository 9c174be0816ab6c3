#!/usr/bin/env python3
"""tools/mfma_classes.py -- per-class effect of the matrix-core tiles on the medium dataset: the lines
re-swept on the final engine (profiles/r03_sweep_medium_mfma.jsonl.gz: cross-row similarity 0.95, >= 20 nonzeros per
row, K = 32 and 128) against the same (line, K) records of the config-3 sweep on the previous build
(profiles/r03_sweep_medium.jsonl.gz).  Markdown on stdout.

  python tools/mfma_classes.py > profiles/r03_mfma_class_summary.md
"""
import gzip
import json
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def load(p):
    op = gzip.open if str(p).endswith(".gz") else open
    out = {}
    for l in op(p, "rt"):
        if l.strip():
            r = json.loads(l)
            out[(r["gen"], r["k"], r.get("dtype", "f64"))] = r
    return out


def main():
    old = load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "profiles" / "r03_sweep_medium.jsonl.gz")
    new = load(sys.argv[2] if len(sys.argv) > 2 else ROOT / "profiles" / "r03_sweep_medium_mfma.jsonl.gz")
    common = [k for k in new if k in old]
    shas = sorted({new[k].get("engine_sha256", "?")[:12] for k in common})
    bad = [k for k in common if not (new[k].get("bitexact_seq_rows", True) and new[k].get("normwise_ok", True))]
    print("### Matrix-core tiles on the medium dataset (final build vs the config-3 build)\n")
    print(f"{len(common)} (line, K) records re-swept on engine build(s) {', '.join(shas)} against "
          f"{old[common[0]].get('engine_sha256', '?')[:12] if common else '-'}; parity failures on the sampled rows: "
          f"{len(bad)}.  Lines: cross-row similarity 0.95, >= 20 nonzeros per row.\n")
    for K in sorted({k[1] for k in common}):
        print(f"#### K = {K}\n")
        print("| avg nnz/row | bw | matrices | with matrix-core tiles | median frac before | median frac after | "
              "aggregate GFLOP/s before | after | speedup geo-mean (tiled lines) | min | max |")
        print("|---|---|---|---|---|---|---|---|---|---|---|")
        cls = defaultdict(list)
        for k in common:
            if k[1] != K:
                continue
            g = k[0].split()
            cls[(int(g[2]), float(g[6]))].append(k)
        allk = []
        for key in sorted(cls):
            ks = cls[key]
            allk += ks
            tiled = [k for k in ks if new[k].get("tile_mode") == "mfma"]
            fb = np.median([old[k]["roofline_frac"] for k in ks])
            fa = np.median([new[k]["roofline_frac"] for k in ks])
            fl = sum(2.0 * new[k]["nnz"] * K for k in ks)
            ab = fl / sum(old[k]["ms"] * 1e-3 for k in ks) / 1e9
            aa = fl / sum(new[k]["ms"] * 1e-3 for k in ks) / 1e9
            if tiled:
                r = np.array([old[k]["ms"] / new[k]["ms"] for k in tiled])
                sp = f"{np.exp(np.log(r).mean()):.3f} | {r.min():.3f} | {r.max():.3f}"
            else:
                sp = "- | - | -"
            print(f"| {key[0]} | {key[1]} | {len(ks)} | {len(tiled)} | {fb:.3f} | {fa:.3f} | {ab:,.0f} | {aa:,.0f} | {sp} |")
        fl = sum(2.0 * new[k]["nnz"] * K for k in allk)
        print(f"| **all** | | {len(allk)} | {sum(new[k].get('tile_mode') == 'mfma' for k in allk)} | "
              f"{np.median([old[k]['roofline_frac'] for k in allk]):.3f} | {np.median([new[k]['roofline_frac'] for k in allk]):.3f} | "
              f"{fl / sum(old[k]['ms'] * 1e-3 for k in allk) / 1e9:,.0f} | {fl / sum(new[k]['ms'] * 1e-3 for k in allk) / 1e9:,.0f} | | | |\n")


if __name__ == "__main__":
    main()
