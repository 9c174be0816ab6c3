#!/usr/bin/env python3
"""tools/generator_fidelity.py -- how closely the synthetic generator reproduces its 11 parameters.

For every generator line of one size of the medium dataset (tools/medium_dataset.py; 1,080 parameter
combinations per size) the matrix is generated and measured with the feature definitions of the reference's
extractor (csr_matrix_features_validation, csr_util_gen.c:889-990; our restatement spmm_host_features is pinned
bit-for-bit to the compiled extractor by tests/test_generator_fidelity.py).  Prints per-feature error statistics
and the worst lines; --jsonl writes one record per line.

The reference generator (artificial-matrix-generator submodule) is absent from the reference tree, so "fidelity"
means: the requested parameter is what the reference's own extractor measures on the output.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
sys.path.insert(0, str(ROOT / "tools"))


def reachable(p: dict, m: int, n: int) -> dict:
    """Targets the extractor can possibly report for the request: skew is capped by the row length limit n
    ((n - avg)/avg), and skew 0 means no imposed heavy row (the natural maximum of the degree distribution)."""
    avg = p["avg"]
    return {"skew_cap": (n - avg) / avg}


def measure(line: str) -> dict:
    import spmm_amd as S
    f = line.split()
    req = {"m": int(f[0]), "n": int(f[1]), "avg": float(f[2]), "std": float(f[3]), "bw": float(f[6]),
           "skew": float(f[7]), "nn": float(f[8]), "crs": float(f[9])}
    A = S.generate(S.gen_params(line))
    ft = S.features(A)
    got = {"avg": ft["avg_nnz_per_row"], "std": ft["std_nnz_per_row"], "bw": ft["avg_bw_scaled"], "skew": ft["skew"],
           "nn": ft["avg_num_neighbours"], "crs": ft["cross_row_similarity"]}
    cap = reachable(req, req["m"], req["n"])["skew_cap"]
    err = {"avg": got["avg"] / req["avg"] - 1.0,
           "bw": got["bw"] / req["bw"] - 1.0,
           "nn": got["nn"] - req["nn"],
           "crs": got["crs"] - req["crs"]}
    if req["skew"] > 0:
        err["skew"] = got["skew"] / min(req["skew"], cap) - 1.0
    else:
        err["std"] = got["std"] / req["std"] - 1.0 if req["std"] > 0 else got["std"] / max(req["avg"], 1e-12)
    return {"gen": line, "req": req, "got": got, "err": err}


def main():
    from spmm_amd.datasets import medium_dataset_lines
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-index", type=int, default=0, help="which matrix size of the dataset (0 = smallest)")
    ap.add_argument("--every", type=int, default=1, help="take every n-th line of that size")
    ap.add_argument("--jsonl", default="")
    ap.add_argument("--worst", type=int, default=8)
    args = ap.parse_args()
    lines = medium_dataset_lines()
    sizes = sorted({(int(l.split()[0]) * (12 * int(l.split()[2]) + 4)) // (1 << 20) for l in lines})
    sel = [l for l in lines if (int(l.split()[0]) * (12 * int(l.split()[2]) + 4)) // (1 << 20) == sizes[args.size_index]]
    sel = sel[::args.every]
    recs = [measure(l) for l in sel]
    if args.jsonl:
        with open(args.jsonl, "w") as fo:
            for r in recs:
                fo.write(json.dumps(r) + "\n")
    print(f"{len(recs)} lines, size {sizes[args.size_index]} MB")
    for key in ("avg", "std", "bw", "skew", "nn", "crs"):
        e = np.array([r["err"][key] for r in recs if key in r["err"]])
        if len(e):
            a = np.abs(e)
            print(f"  {key:5s} n={len(e):5d} median|err|={np.median(a):.4f} p90={np.percentile(a, 90):.4f} "
                  f"max={a.max():.4f} mean={e.mean():+.4f}")
    for key in ("bw", "nn", "crs", "skew"):
        worst = sorted((r for r in recs if key in r["err"]), key=lambda r: -abs(r["err"][key]))[:args.worst]
        print(f"worst {key}:")
        for r in worst:
            print(f"   {r['err'][key]:+.4f}  {r['gen']}  got {r['got'][key]:.4f}")


if __name__ == "__main__":
    main()
