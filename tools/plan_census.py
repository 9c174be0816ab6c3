#!/usr/bin/env python3
"""tools/plan_census.py -- the matrix-core gate over the whole medium dataset, on the host (no GPU).

For every generator line of synthetic_matrices_medium_dataset (spmm_amd.datasets) and every K: the engine's own
inspector (spmm_hip_debug_plan, gate-only mode) decides whether the matrix runs matrix-core tiles.  The gate reads
only its sampled 16-row tiles (spmm_amd.gate_sample_rows), so the matrix is generated for those rows only
(spmm_host_generate_masked: same rows, bit for bit, as the full generation).  One JSON line per (line, K): the
decision, the gate's sample statistics and cost model, the split length and panel width, tagged with the engine
fingerprint (bench.engine_sha256).  Resumable: (line, K) pairs already in --out for this engine are skipped.

A line whose decision is "mfma" is planned differently from the engine without matrix-core tiles (SPMM_HIP_MFMA=-1,
the plan of the config-3 sweep build b4d29bad); every other line's plan is unchanged (tests/test_census.py checks
the plan fingerprints on a sample).  tools/sessions/r04_sweep.sh re-measures exactly the changed (line, K) pairs
(profiles/r04/changed_pairs.txt, written by `--pairs-out`) against the plan without matrix-core tiles.

  python tools/plan_census.py --k 32,128 --workers 6 --out /tmp/plan_census.jsonl
  python tools/plan_census.py --out /tmp/plan_census.jsonl --regate-out profiles/r04/plan_census.jsonl \
      --pairs-out profiles/r04/changed_pairs.txt        # then gzip: profiles/r04/plan_census.jsonl.gz
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
sys.path.insert(0, str(ROOT))

KEEP = ("mode", "gate", "r16", "take", "est_tiles", "est_tile_nnz", "est_chunks", "max_chunks", "t_on_us", "t_off_us",
        "sampled", "seq_max", "kw", "npanels")


def census_line(job):
    idx, line, ks, sha = job
    import numpy as np
    import spmm_amd as S
    p = S.gen_params(line)
    t0 = time.time()
    A = S.generate_masked(p, S.gate_sample_rows(int(p.nr_rows)))
    t_gen = time.time() - t0
    out = []
    for k in ks:
        d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64, 0, gate_only=True)
        rec = {"idx": idx, "gen": line, "k": k, "m": int(A.m), "ncols": int(A.ncols), "nnz": int(A.nnz),
               "engine_sha256": sha, "gen_s": round(t_gen, 3)}
        rec.update({f: (round(d[f], 5) if isinstance(d[f], float) else d[f]) for f in KEEP})
        out.append(rec)
    del A
    return out


def regate(args):
    """Re-decide every record of --out with THIS library's gate constants (spmm_hip_debug_gate on the recorded gate
    sample -- the sample itself comes from the engine's mfma_sample, unchanged), stamp this engine build, write
    --regate-out and the changed pairs (--pairs-out)."""
    import bench
    import spmm_amd as S
    sha = bench.engine_sha256()
    recs = [json.loads(l) for l in Path(args.out).read_text().splitlines()]
    pairs = []
    with open(args.regate_out, "w") as f:
        for r in recs:
            g = S.debug_gate(r["m"], r["nnz"], r["k"], r)
            r.update({"gate": g["gate"], "t_on_us": round(g["t_on_us"], 5), "t_off_us": round(g["t_off_us"], 5),
                      "mode": "mfma" if g["gate"] else "none", "engine_sha256": sha, "sampled_by": r["engine_sha256"]})
            f.write(json.dumps(r) + "\n")
            if g["gate"]:
                pairs.append(f"{r['k']}\t{r['gen']}")
    if args.pairs_out:
        Path(args.pairs_out).write_text("\n".join(sorted(set(pairs))) + "\n")
    print(f"{args.regate_out}: {len(recs)} records, {len(set(pairs))} (line, K) pairs take matrix-core tiles")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", default="32,128")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--threads", type=int, default=2, help="OpenMP threads per worker (the generator)")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--budget", type=float, default=1e9)
    ap.add_argument("--order-by", default=None, help="an earlier census: lines in decreasing sampled reuse")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04" / "plan_census.jsonl"))
    ap.add_argument("--pairs-out", default=None, help="write 'K<TAB>line' of every mfma (line, K) of this engine here")
    ap.add_argument("--regate-out", default=None,
                    help="re-decide the records of --out with this library's gate (no generation) into this file")
    args = ap.parse_args()
    if args.regate_out:
        return regate(args)
    os.environ["OMP_NUM_THREADS"] = str(args.threads)
    import bench
    from spmm_amd.datasets import medium_dataset_lines
    sha = bench.engine_sha256()
    ks = [int(x) for x in args.k.split(",")]
    out = Path(args.out)
    done = set()
    if out.exists():
        for l in out.read_text().splitlines():
            d = json.loads(l)
            if d.get("engine_sha256") == sha:
                done.add((d["gen"], d["k"]))
    lines = medium_dataset_lines()
    jobs = []
    for i in range(args.offset, len(lines), args.stride):
        todo = [k for k in ks if (lines[i], k) not in done]
        if todo:
            jobs.append((i, lines[i], todo, sha))
    if args.order_by and Path(args.order_by).exists():
        # likely-changed lines first (highest sampled reuse of an earlier census), so the changed set is known early
        prev = {}
        for l in Path(args.order_by).read_text().splitlines():
            d = json.loads(l)
            prev[d["gen"]] = max(prev.get(d["gen"], 0.0), float(d.get("r16", 0.0)))
        jobs.sort(key=lambda j: -prev.get(j[1], 0.0))
    print(f"{len(jobs)} lines to do ({len(done)} (line, K) done)", flush=True)
    from multiprocessing import get_context
    t0 = time.time()
    n = 0
    with get_context("fork").Pool(args.workers, maxtasksperchild=50) as pool, open(out, "a") as f:
        for recs in pool.imap(census_line, jobs, chunksize=1):
            for r in recs:
                f.write(json.dumps(r) + "\n")
            f.flush()
            n += 1
            if n % 200 == 0:
                print(f"{n}/{len(jobs)} lines, {time.time() - t0:.0f} s", flush=True)
            if time.time() - t0 > args.budget:
                pool.terminate()
                break
    print(f"done: {n} lines in {time.time() - t0:.0f} s", flush=True)
    if args.pairs_out:
        pairs = []
        for l in out.read_text().splitlines():
            d = json.loads(l)
            if d.get("engine_sha256") == sha and d.get("mode") == "mfma":
                pairs.append(f"{d['k']}\t{d['gen']}")
        Path(args.pairs_out).write_text("\n".join(sorted(set(pairs))) + "\n")
        print(f"{args.pairs_out}: {len(set(pairs))} changed (line, K) pairs", flush=True)


if __name__ == "__main__":
    main()
