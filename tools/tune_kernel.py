#!/usr/bin/env python3
"""tools/tune_kernel.py -- A/B the row-kernel variants of the tuning build on the benchmark matrix (MI355X).

Loads lib/libspmm_hip_tune.so (built with -DSPMM_TUNING: a grid of K=32 fp64 row-kernel variants), runs every
variant on the same HBM-resident A, B, C, interleaved over several rounds in ONE process (cdna_hip_programming.md
§5.4 rule 24), and prints per-variant median / min launch time (HIP events on the launch stream) and whether the
output is bit-identical to the first variant.  Output: one JSON line per variant + a summary, to stdout.
"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))

# (U, NTC, DMA, BUF, seq_max, cap, panel_k[, win_bytes[, xcd]]): 0 = inspector policy default (win_bytes -1 = no
# windows; xcd 1 = XCD-contiguous block order, -1 = off)
VARIANTS = [(16, 1, 0, 1, 0, 0, 0), (16, 1, 1, 1, 0, 0, 0), (16, 1, 0, 0, 0, 0, 0), (8, 1, 0, 1, 0, 0, 0),
            (16, 1, 0, 1, 2048, 0, 0), (16, 1, 0, 1, 64, 0, 0), (16, 1, 0, 1, 128, 0, 0), (16, 1, 0, 1, 256, 0, 0),
            (16, 1, 0, 1, 512, 0, 0), (16, 1, 0, 1, 0, 1024, 0), (16, 1, 0, 1, 0, 2048, 0), (16, 1, 0, 1, 0, 4096, 0),
            (16, 1, 0, 1, 0, 0, 16), (16, 1, 0, 1, 0, 0, 64), (16, 1, 0, 1, 0, 0, 4096)]
FIELDS = ("U", "NTC", "DMA", "BUF", "SEQ_MAX", "CAP", "PANEL_K", "WIN_BYTES", "XCD", "LANES")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gen", default="1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14")
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="", help="comma list of variant indices")
    ap.add_argument("--variants", default="", help="';'-separated U,NTC,DMA,BUF,SEQ_MAX,CAP,PANEL_K tuples")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    args = ap.parse_args()

    import torch
    import spmm_amd as S
    T = S._bind_hip(C.CDLL(str(ROOT / "spmm-research_amd" / "lib" / "libspmm_hip_tune.so")))
    T.spmm_hip_tune_select.argtypes = [C.c_void_p] + [C.c_int] * 7 + [C.c_int64, C.c_int, C.c_int]

    A = S.generate(S.gen_params(args.gen))
    k = args.k
    h = C.c_void_p()
    vals = A.values if args.dtype == "f64" else A.values.astype(np.float32)
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    st = T.spmm_hip_create(A.row_ptr, A.col_idx, vals.ctypes.data_as(C.c_void_p), A.m, A.ncols, A.nnz, k,
                           S.F64 if args.dtype == "f64" else S.F32, 0, C.byref(h))
    assert st == 0, (st, T.spmm_hip_last_error_detail())
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=tdt)
    Cm = torch.empty((A.m, k), device=dev, dtype=tdt)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)

    variants = VARIANTS if not args.only else [VARIANTS[int(i)] for i in args.only.split(",")]
    if args.variants:
        variants = [tuple(int(x) for x in v.split(",")) for v in args.variants.split(";")]
    variants = [tuple(v) + (0,) * (10 - len(v)) for v in variants]
    bytes_alg = S.bytes_alg(A.m, A.ncols, A.nnz, k, S.F64 if args.dtype == "f64" else S.F32)
    ref = None
    res = {v: [] for v in variants}
    same = {}
    plan = {}
    for rnd in range(args.rounds):
        for v in variants:
            assert T.spmm_hip_tune_select(h, *v) == 0, T.spmm_hip_last_error_detail()
            for _ in range(2):
                T.spmm_hip_run_device(h, C.c_void_p(B.data_ptr()), S.B_ROW_MAJOR, C.c_void_p(Cm.data_ptr()), k, sp)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                T.spmm_hip_run_device(h, C.c_void_p(B.data_ptr()), S.B_ROW_MAJOR, C.c_void_p(Cm.data_ptr()), k, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / args.iters)
            if rnd == 0:
                inf = np.zeros(S.INFO_SLOTS, np.int64)
                T.spmm_hip_info(h, inf)
                plan[v] = {"T": int(inf[8]), "cap": int(inf[9]), "panel_k": int(inf[10]), "blocks": int(inf[5]),
                           "split_rows": int(inf[6]), "windows": int(inf[12]), "win_cols": int(inf[13]),
                           "segments": int(inf[14]), "xcd": int(inf[15]), "lmax": int(inf[16]),
                           "exact_rows": int(inf[17])}
                out = Cm.clone()
                if ref is None:
                    ref = out
                # equal up to split-row rounding: rows <= min T are bitwise equal across variants
                same[v] = bool(torch.allclose(out, ref, rtol=1e-12, atol=0))
    rows = []
    for v in variants:
        t = np.array(res[v])
        rows.append({"variant": dict(zip(FIELDS, v)), "median_ms": float(np.median(t)),
                     "min_ms": float(t.min()), "gbs_alg": bytes_alg / (np.median(t) * 1e-3) / 1e9,
                     "close": same[v], "plan": plan[v]})
        print(json.dumps(rows[-1]), flush=True)
    best = min(rows, key=lambda r: r["median_ms"])
    print(json.dumps({"best": best, "matrix": args.gen, "k": k, "dtype": args.dtype, "nnz": int(A.nnz)}), flush=True)
    T.spmm_hip_destroy(h)


if __name__ == "__main__":
    main()
