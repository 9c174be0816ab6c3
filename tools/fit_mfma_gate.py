#!/usr/bin/env python3
"""tools/fit_mfma_gate.py -- fit the matrix-core gate's cost model (spmm_engine.hip mfma_cost) on
same-process A/B measurements.

  features   the gate's sample (spmm_hip_debug_plan, gate-only, on the sampled rows) of every line in an A/B file,
             with the A/B run's tile selection (--npc, SPMM_HIP_MFMA_NPC), for K in the records
  fit        least squares of the model's constants on the measured times: the tile kernel (launch + per chunk +
             per tile, or the longest tile's chain) and the row kernel (launch + per nonzero and 32-column panel),
             then the decision threshold; prints the constants and the A/B outcome of the resulting gate per class

  python tools/fit_mfma_gate.py features --ab gpurun_out/r04c/fit_ab*.jsonl --npc 96 --out profiles/r04/fit_features.jsonl
  python tools/fit_mfma_gate.py fit --ab ... --features profiles/r04/fit_features.jsonl
"""
import argparse
import glob
import json
import math
import os
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def load_ab(patterns):
    recs = {}
    for pat in patterns:
        for f in glob.glob(pat):
            for l in open(f):
                if l.startswith("{"):
                    d = json.loads(l)
                    if "ms_base" in d:
                        recs[(d["gen"], d["k"])] = d
    return recs


def feat_job(job):
    line, ks, npc = job
    os.environ["SPMM_HIP_MFMA_NPC"] = str(npc)
    import spmm_amd as S
    p = S.gen_params(line)
    A = S.generate_masked(p, S.gate_sample_rows(int(p.nr_rows)))
    out = []
    for k in ks:
        d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64, 2, gate_only=True)
        out.append({"gen": line, "k": k, "m": int(A.m), "nnz": int(A.nnz), "npc": npc,
                    **{f: d[f] for f in ("sampled", "r16", "take", "est_tiles", "est_tile_nnz", "est_chunks",
                                         "max_chunks", "seq_max", "kw")}})
    return out


def features(args):
    lines = defaultdict(list)
    if args.lines:
        for g in Path(args.lines).read_text().splitlines():
            if g.strip():
                lines[g.strip()] = [int(x) for x in args.k.split(",")]
    else:
        for (g, k) in load_ab(args.ab):
            lines[g].append(k)
    os.environ["OMP_NUM_THREADS"] = str(args.threads)
    from multiprocessing import get_context
    with get_context("fork").Pool(args.workers) as pool, open(args.out, "w") as f:
        for recs in pool.imap_unordered(feat_job, [(g, sorted(ks), args.npc) for g, ks in lines.items()]):
            for r in recs:
                f.write(json.dumps(r) + "\n")
    print(f"{args.out}: {sum(len(v) for v in lines.values())} (line, K)")


def model(F, c):
    """t_on, t_off (us) for feature rows F with constants c (mirrors mfma_cost)."""
    P = F["k"] / 32.0
    r_row = c["row_us_nnz"] * np.maximum(F["r16"], 1.0) ** -c["row_reuse_exp"] * (F["kw"] / 32.0) ** -c["row_kw_exp"]
    t_off = c["launch"] + F["nnz"] * P * r_row
    t_tiles = c["launch"] + P * np.maximum(F["est_chunks"] * c["us_chunk"] + F["est_tiles"] * c["us_tile"],
                                           F["max_chunks"] * c["us_chain"])
    t_left = c["launch"] + (F["nnz"] - F["est_tile_nnz"]) * P * r_row
    return np.maximum(t_tiles, t_left), t_off


def fit(args):
    ab = load_ab(args.ab)
    feats = {}
    for l in open(args.features):
        d = json.loads(l)
        feats[(d["gen"], d["k"])] = d
    keys = [k for k in ab if k in feats and ab[k]["tile_mode"] == "mfma"]
    F = {f: np.array([feats[k][f] if f in feats[k] else ab[k][f] for k in keys], float)
         for f in ("k", "nnz", "est_chunks", "est_tiles", "est_tile_nnz", "max_chunks", "r16", "kw")}
    t_on = np.array([ab[k]["ms"] * 1e3 for k in keys])
    t_off = np.array([ab[k]["ms_base"] * 1e3 for k in keys])
    P = F["k"] / 32.0
    from scipy.optimize import least_squares
    # row kernel: t_off = launch + r * nnz * P (relative error)
    def res_off(x):
        c = {"launch": x[0], "row_us_nnz": x[1], "row_reuse_exp": x[2], "row_kw_exp": x[3], "us_chunk": 1.0,
             "us_tile": 0.0, "us_chain": 0.0}
        return np.log(model(F, c)[1] / t_off)
    r0 = least_squares(res_off, [10.0, 12e-6, 0.1, 0.1], bounds=([0, 0, -1, -1], [100, 1e-3, 2, 2])).x
    # the shipped time: max(tile kernel, leftover rows) with the tile kernel's launch + max(throughput, chain)
    def res_on(x):
        c = {"launch": r0[0], "row_us_nnz": r0[1], "row_reuse_exp": r0[2], "row_kw_exp": r0[3], "us_chunk": x[0],
             "us_tile": x[1], "us_chain": x[2]}
        m_on, _ = model(F, c)
        return np.log(m_on / t_on)
    x = least_squares(res_on, [1.6e-3, 1e-3, 4.5], bounds=([0, 0, 0], [1e-2, 1e-2, 50]), loss="soft_l1").x
    c = {"launch": float(r0[0]), "row_us_nnz": float(r0[1]), "row_reuse_exp": float(r0[2]),
         "row_kw_exp": float(r0[3]), "us_chunk": float(x[0]), "us_tile": float(x[1]), "us_chain": float(x[2])}
    m_on, m_off = model(F, c)
    print(json.dumps({"fit": c, "lines": len(keys),
                      "rms_log_err_on": float(np.sqrt(np.mean(np.log(m_on / t_on) ** 2))),
                      "rms_log_err_off": float(np.sqrt(np.mean(np.log(m_off / t_off) ** 2)))}))
    m_on, m_off = model(F, c)
    sp = t_off / t_on
    pred = m_off / m_on
    for thr in (1.0, 1.05, 1.1, 1.15, 1.2, 1.3):
        on = pred >= thr
        tot_off, tot_chosen = t_off.sum(), np.where(on, t_on, t_off).sum()
        print(json.dumps({"gain_threshold": thr, "taken": int(on.sum()), "worst_taken": float(sp[on].min()) if on.any() else None,
                          "taken_below_0.9": int((sp[on] < 0.9).sum()), "taken_below_1.0": int((sp[on] < 1.0).sum()),
                          "missed_above_1.1": int((sp[~on] > 1.1).sum()), "aggregate_speedup": round(tot_off / tot_chosen, 4)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["features", "fit"])
    ap.add_argument("--ab", nargs="+", default=[])
    ap.add_argument("--features", default=str(ROOT / "profiles" / "r04" / "fit_features.jsonl"))
    ap.add_argument("--npc", type=float, default=96.0)
    ap.add_argument("--lines", default=None, help="features: a file of generator lines instead of --ab")
    ap.add_argument("--k", default="32,128")
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04" / "fit_features.jsonl"))
    args = ap.parse_args()
    {"features": features, "fit": fit}[args.mode](args)


if __name__ == "__main__":
    main()
