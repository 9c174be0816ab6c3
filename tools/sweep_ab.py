#!/usr/bin/env python3
"""tools/sweep_ab.py -- compare the kernel times of two sets of sweep records on their common (line, K, dtype).

Used to show that the parallel host workers of tools/sweep.py (timed regions under an exclusive lock, ms = the lowest
of 3 batch means) reproduce the single-process sweep's times: prints, per K, the median / p10 / p90 of ms(B) / ms(A)
and the count of records off by more than 10 %.

  python tools/sweep_ab.py profiles/r03_sweep_medium.jsonl.gz 'gpurun_out/sweep/ab_par3.w*.jsonl'
"""
import argparse
import glob
import gzip
import json

import numpy as np


def load(pattern):
    recs = {}
    for p in sorted(glob.glob(pattern)):
        op = gzip.open if p.endswith(".gz") else open
        with op(p, "rt") as f:
            for line in f:
                if line.startswith("{"):
                    r = json.loads(line)
                    recs[(r["gen"], r["k"], r.get("dtype", "f64"))] = r
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a", help="reference records (glob)")
    ap.add_argument("b", help="records to compare (glob)")
    ap.add_argument("--min-ms", type=float, default=0.0, help="only records whose reference time is at least this")
    args = ap.parse_args()
    A, B = load(args.a), load(args.b)
    common = [k for k in B if k in A and A[k]["ms"] >= args.min_ms]
    print(f"{len(common)} common records ({len(A)} in A, {len(B)} in B)\n")
    print("| K | records | median B/A | p10 | p90 | off > 10 % | worst |")
    print("|---|---|---|---|---|---|---|")
    allr = []
    for k in sorted({c[1] for c in common}):
        r = np.array([B[c]["ms"] / A[c]["ms"] for c in common if c[1] == k])
        allr.append(r)
        print(f"| {k} | {len(r)} | {np.median(r):.3f} | {np.percentile(r, 10):.3f} | {np.percentile(r, 90):.3f} | "
              f"{int((np.abs(r - 1) > 0.1).sum())} | {r[np.argmax(np.abs(np.log(r)))]:.2f} |")
    if allr:
        r = np.concatenate(allr)
        print(f"| all | {len(r)} | {np.median(r):.3f} | {np.percentile(r, 10):.3f} | {np.percentile(r, 90):.3f} | "
              f"{int((np.abs(r - 1) > 0.1).sum())} | {r[np.argmax(np.abs(np.log(r)))]:.2f} |")


if __name__ == "__main__":
    main()
