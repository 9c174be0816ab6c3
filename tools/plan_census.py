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
the plan fingerprints on a sample).  tools/mfma_ab.py --census re-measures exactly the changed lines.

  python tools/plan_census.py --k 32,128 --workers 6 --out profiles/r04_plan_census.jsonl
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", default="32,128")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--threads", type=int, default=2, help="OpenMP threads per worker (the generator)")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--budget", type=float, default=1e9)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04_plan_census.jsonl"))
    args = ap.parse_args()
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
    # small matrices first would leave the big ones for last; interleave by size so progress is steady
    print(f"{len(jobs)} lines to do ({len(done)} (line, K) done)", flush=True)
    from multiprocessing import get_context
    t0 = time.time()
    n = 0
    with get_context("fork").Pool(args.workers, maxtasksperchild=50) as pool, open(out, "a") as f:
        for recs in pool.imap_unordered(census_line, jobs, chunksize=1):
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


if __name__ == "__main__":
    main()
