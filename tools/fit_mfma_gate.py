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


def load_ab(patterns, dtype="f64"):
    recs = {}
    for pat in patterns:
        for f in glob.glob(pat):
            for l in open(f):
                if l.startswith("{"):
                    d = json.loads(l)
                    if "ms_base" in d and d.get("dtype", "f64") == dtype:
                        recs[(d["gen"], d["k"])] = d
    return recs


def feat_job(job):
    line, ks, npc, dtype = job
    os.environ["SPMM_HIP_MFMA_NPC"] = str(npc)
    import spmm_amd as S
    p = S.gen_params(line)
    A = S.generate_masked(p, S.gate_sample_rows(int(p.nr_rows)))
    out = []
    for k in ks:
        d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64 if dtype == "f64" else S.F32, 2, gate_only=True)
        out.append({"gen": line, "k": k, "dtype": dtype, "m": int(A.m), "nnz": int(A.nnz), "npc": npc,
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
        for (g, k) in load_ab(args.ab, args.dtype):
            lines[g].append(k)
    os.environ["OMP_NUM_THREADS"] = str(args.threads)
    from multiprocessing import get_context
    with get_context("fork").Pool(args.workers) as pool, open(args.out, "w") as f:
        for recs in pool.imap_unordered(feat_job, [(g, sorted(ks), args.npc, args.dtype) for g, ks in lines.items()]):
            for r in recs:
                f.write(json.dumps(r) + "\n")
    print(f"{args.out}: {sum(len(v) for v in lines.values())} (line, K)")


def model(F, c):
    """t_on, t_off (us) for feature rows F with constants c (mirrors mfma_cost in spmm_engine.hip)."""
    P = F["k"] / 32.0
    r_row = c["row_us_nnz"] * np.maximum(F["r16"], 1.0) ** -c["row_reuse_exp"] * (F["kw"] / 32.0) ** -c["row_kw_exp"]
    t_off = c["launch"] + P * (F["nnz"] * r_row + F["m"] * c["row_us_row"])
    # + the per-launch exact-range check of B (one pass over ncols x K values; square dataset matrices: ncols = m)
    b_mb = F["m"] * F["k"] * F.get("vsize", 8.0) / 1e6
    t_tiles = c["mfma_launch"] + P * np.maximum(F["est_chunks"] * c["us_chunk"] + F["est_tiles"] * c["us_tile"],
                                                F["max_chunks"] * c["us_chain"]) + b_mb * c.get("us_bmb", 0.0)
    left_rows = np.maximum(F["m"] - 16.0 * F["est_tiles"], 0.0)
    t_left = c["launch"] + P * ((F["nnz"] - F["est_tile_nnz"]) * r_row + left_rows * c["row_us_row"])
    return np.maximum(t_tiles, t_left), t_off


def decide(F, c):
    """The gate: tiles hold at least MIN_TILE_FRAC of the nonzeros, the model's gain reaches c["gain"], and with one
    32-column sub-panel (K < 64) rows average at least c["k32_min_row_nnz"] nonzeros."""
    m_on, m_off = model(F, c)
    return ((F["est_tile_nnz"] >= c["min_tile_frac"] * F["nnz"]) & (F["est_tiles"] > 0) & (m_off >= c["gain"] * m_on) &
            ((F["k"] >= 64) | (F["nnz"] >= c.get("k32_min_row_nnz", 0.0) * F["m"])))


def fit(args):
    from scipy.optimize import least_squares
    ab = load_ab(args.ab, args.dtype)
    feats = {}
    for l in open(args.features):
        d = json.loads(l)
        if d.get("dtype", "f64") == args.dtype:
            feats[(d["gen"], d["k"])] = d
    keys = [k for k in ab if k in feats and ab[k]["tile_mode"] == "mfma"]
    F = {f: np.array([feats[k][f] if f in feats[k] else ab[k][f] for k in keys], float)
         for f in ("k", "nnz", "m", "est_chunks", "est_tiles", "est_tile_nnz", "max_chunks", "r16", "kw")}
    F["vsize"] = np.full(len(keys), 8.0 if args.dtype == "f64" else 4.0)
    t_on = np.array([ab[k]["ms"] * 1e3 for k in keys])
    t_off = np.array([ab[k]["ms_base"] * 1e3 for k in keys])
    base = {"min_tile_frac": 0.0, "gain": 1.0}

    def c_of(x, y):
        return {**base, "launch": y[0], "row_us_nnz": y[1], "row_reuse_exp": y[2], "row_kw_exp": y[3],
                "row_us_row": y[4], "mfma_launch": x[0], "us_chunk": x[1], "us_tile": x[2], "us_chain": x[3],
                "us_bmb": x[4] if len(x) > 4 else 0.0}
    # the row kernel (every line: the baseline plan has no matrix-core tiles)
    y = least_squares(lambda y: np.log(model(F, c_of([0, 0, 0, 0, 0], y))[1] / t_off), [5, 2.5e-5, 0.2, 0.15, 1e-4],
                      bounds=([0, 0, -2, -2, 0], [100, 1e-3, 3, 3, 1e-2])).x
    # the tile kernel on the lines whose tiles hold >= 90 % of the nonzeros (t_on is then the tile kernel)
    sel = F["est_tile_nnz"] >= 0.9 * F["nnz"]
    Fs = {k: v[sel] for k, v in F.items()}
    x = least_squares(lambda x: np.log(model(Fs, c_of(x, y))[0] / t_on[sel]), [20, 1.6e-3, 1.5e-3, 1.1, 0.2],
                      bounds=([0, 0, 0, 0, 0], [200, 1e-2, 1e-2, 50, 5]), loss="soft_l1").x
    c = c_of(x, y)
    m_on, m_off = model(F, c)
    print(json.dumps({"fit": {k: float(v) for k, v in c.items()}, "lines": len(keys), "tile_lines": int(sel.sum()),
                      "rms_log_err_on_tile_lines": float(np.sqrt(np.mean(np.log(m_on[sel] / t_on[sel]) ** 2))),
                      "rms_log_err_off": float(np.sqrt(np.mean(np.log(m_off / t_off) ** 2)))}))
    sp = t_off / t_on
    cls = [(k[1], k[0].split()[2], k[0].split()[9]) for k in keys]
    for frac in (0.0, 0.8, 0.9):
        for thr in (1.1, 1.2, 1.3, 1.4):
            cc = {**c, "min_tile_frac": frac, "gain": thr}
            on = decide(F, cc)
            chosen = np.where(on, t_on, t_off)
            worst_cls = min((t_off[[i for i in range(len(keys)) if cls[i] == q and on[i]]].sum() /
                             t_on[[i for i in range(len(keys)) if cls[i] == q and on[i]]].sum(), q)
                            for q in set(cls) if any(on[i] for i in range(len(keys)) if cls[i] == q))
            print(json.dumps({"min_tile_frac": frac, "gain": thr, "taken": int(on.sum()),
                              "worst_line": round(float(sp[on].min()), 3) if on.any() else None,
                              "below_0.9": int((sp[on] < 0.9).sum()), "below_1.0": int((sp[on] < 1.0).sum()),
                              "missed_above_1.2": int((sp[~on] > 1.2).sum()),
                              "worst_class_taken": [round(float(worst_cls[0]), 3), worst_cls[1]],
                              "aggregate": round(float(t_off.sum() / chosen.sum()), 4)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["features", "fit"])
    ap.add_argument("--ab", nargs="+", default=[])
    ap.add_argument("--features", default=str(ROOT / "profiles" / "r04" / "fit_features.jsonl"))
    ap.add_argument("--npc", type=float, default=96.0)
    ap.add_argument("--lines", default=None, help="features: a file of generator lines instead of --ab")
    ap.add_argument("--k", default="32,128")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64", help="the A/B records' and the gate's value type")
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04" / "fit_features.jsonl"))
    args = ap.parse_args()
    {"features": features, "fit": fit}[args.mode](args)


if __name__ == "__main__":
    main()
