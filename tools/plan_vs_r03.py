#!/usr/bin/env python3
"""tools/plan_vs_r03.py -- is the engine's plan WITHOUT matrix-core tiles still the plan of the config-3 sweep build
(engine b4d29bad, profiles/r03_sweep_medium.jsonl.gz)?  For a stride sample of the dataset lines (every --stride-th,
up to --max-nnz nonzeros) and every K the sweep recorded, the host planner (spmm_hip_debug_plan, SPMM_HIP_MFMA=-1
plan) must reproduce the recorded plan: split length, K panel width, split rows, row blocks, exact rows, vector
lanes, XCD order, column windows and LDS tiles.  Prints one JSON summary (and every mismatch).

  python tools/plan_vs_r03.py --stride 97 --max-nnz 2e7 --workers 6
"""
import argparse
import gzip
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
R03 = ROOT / "profiles" / "r03_sweep_medium.jsonl.gz"
# recorded field -> debug_plan field
FIELDS = {"seq_max": "seq_max", "panel_k": "kw", "split_rows": "split_rows", "blocks": "blocks",
          "exact_rows": "exact_rows", "lmax": "lmax", "xcd": "xcd", "windows": "nwin", "tiles": "ntile"}


def r03_records(stride, max_nnz):
    by_line = defaultdict(dict)
    for l in gzip.open(R03, "rt"):
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        if d["idx"] % stride == 0 and d["nnz"] <= max_nnz and d.get("dtype", "f64") == "f64":
            by_line[d["gen"]][d["k"]] = {f: d[f] for f in FIELDS}
    return by_line


def check_line(job):
    line, recs = job
    import spmm_amd as S
    A = S.generate(S.gen_params(line))
    out = []
    for k, rec in sorted(recs.items()):
        d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64, -1)
        bad = {f: (rec[f], int(d[g])) for f, g in FIELDS.items() if int(rec[f]) != int(d[g])}
        out.append((line, k, bad))
    return out


def compare(stride=97, max_nnz=2e7, workers=4):
    jobs = sorted(r03_records(stride, max_nnz).items())
    res = []
    if workers > 1:
        from multiprocessing import get_context
        with get_context("fork").Pool(workers) as pool:
            for r in pool.imap_unordered(check_line, jobs):
                res += r
    else:
        for j in jobs:
            res += check_line(j)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stride", type=int, default=97)
    ap.add_argument("--max-nnz", type=float, default=2e7)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--threads", type=int, default=2)
    args = ap.parse_args()
    os.environ["OMP_NUM_THREADS"] = str(args.threads)
    res = compare(args.stride, args.max_nnz, args.workers)
    bad = [r for r in res if r[2]]
    for line, k, b in bad:
        print(json.dumps({"gen": line, "k": k, "mismatch": b}))
    print(json.dumps({"lines": len({r[0] for r in res}), "pairs": len(res), "mismatched_pairs": len(bad),
                      "stride": args.stride, "max_nnz": args.max_nnz}))


if __name__ == "__main__":
    main()
