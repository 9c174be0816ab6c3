#!/usr/bin/env python3
"""tools/ab_tiles.py -- A/B of the LDS B tile mode (spmm_tile_kernel) against the row kernel on MI355X.

For each generator line x K x dtype: one handle per mode (SPMM_HIP_TILES=-1 row kernel only, 0 = policy, 1 = every
eligible tile), the same HBM-resident B, launches interleaved over rounds in one process; HIP events on the launch
stream; median ms per mode; the rows both modes report exact must be bit-identical.  One JSON line per case.
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))

LINES = ["39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14",
         "22354 22354 500 166.6667 normal random 0.05 100 0.05 0.05 14",
         "22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14",
         "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14",
         "111476 111476 100 33.3333 normal random 0.6 1000 1.9 0.5 14",
         "222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14",
         "550072 550072 20 6.6667 normal random 0.6 1000 0.5 0.95 14",
         "1082401 1082401 10 3.3333 normal random 0.6 100 0.95 0.95 14",
         "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", default="", help="';'-separated generator lines (default: a built-in set)")
    ap.add_argument("--k", default="32")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--modes", default="-1,0,1",
                    help="SPMM_HIP_TILES values; a 'w<S>' suffix (e.g. 1w2) sets SPMM_HIP_TILE_WIDE=<S>, others get 1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--env", default="", help="extra KEY=VAL;KEY=VAL for the tile handles")
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    lines = args.lines.split(";") if args.lines else LINES
    modes = args.modes.split(",")
    extra = dict(kv.split("=", 1) for kv in args.env.split(";") if kv)
    for line in lines:
        A = S.generate(S.gen_params(line))
        for k in (int(x) for x in args.k.split(",")):
            for dt in args.dtype.split(","):
                npdt = np.float64 if dt == "f64" else np.float32
                tdt = torch.float64 if dt == "f64" else torch.float32
                vals = A.values.astype(npdt)
                hs = {}
                for md in modes:
                    tm, _, sw = md.partition("w")
                    os.environ["SPMM_HIP_TILES"] = tm
                    os.environ["SPMM_HIP_TILE_WIDE"] = sw or "1"
                    for kk, vv in extra.items():
                        if int(tm) >= 0:
                            os.environ[kk] = vv
                        else:
                            os.environ.pop(kk, None)
                    hs[md] = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
                os.environ.pop("SPMM_HIP_TILES", None)
                os.environ.pop("SPMM_HIP_TILE_WIDE", None)
                for kk in extra:
                    os.environ.pop(kk, None)
                g = torch.Generator(device=dev)
                g.manual_seed(42)
                B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=tdt)
                Cs = {md: torch.empty((A.m, k), device=dev, dtype=tdt) for md in modes}
                times = {md: [] for md in modes}
                for rnd in range(args.rounds):
                    for md in modes:
                        mf, Cm = hs[md], Cs[md]
                        for _ in range(2):
                            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cm.data_ptr(), k, stream.cuda_stream)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(stream)
                        for _ in range(args.iters):
                            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cm.data_ptr(), k, stream.cuda_stream)
                        e1.record(stream)
                        torch.cuda.synchronize()
                        times[md].append(e0.elapsed_time(e1) / args.iters)
                ref = modes[0]
                ex0 = hs[ref].exact_rows()
                c0 = Cs[ref].cpu().numpy()
                iv = np.int64 if dt == "f64" else np.int32
                out = {"gen": line, "k": k, "dtype": dt, "nnz": A.nnz}
                for md in modes:
                    med = float(np.median(times[md]))
                    ti = hs[md].tile_info()
                    exm = hs[md].exact_rows() & ex0
                    cm = Cs[md].cpu().numpy()
                    same = bool(np.array_equal(cm[exm].view(iv), c0[exm].view(iv)))
                    fin = bool(np.isfinite(cm).all())
                    b = S.bytes_alg(A.m, A.ncols, A.nnz, k, S.F64 if dt == "f64" else S.F32)
                    out[str(md)] = {"ms": round(med, 5), "gflops": round(2.0 * A.nnz * k / med / 1e6, 1),
                                    "frac": round(b / (med * 1e-3) / 8e12, 4), "tiles": ti["tiles"],
                                    "tile_rows": ti["rows"], "tile_nnz": ti["nnz"], "chunks": ti["chunks"],
                                    "reuse": ti["reuse"], "wide": ti["wide"], "exact_same": same, "finite": fin}
                base = out[str(ref)]["ms"]
                for md in modes:
                    out[str(md)]["speedup"] = round(base / out[str(md)]["ms"], 3)
                print(json.dumps(out), flush=True)
                for mf in hs.values():
                    mf.close()
                del B, Cs


if __name__ == "__main__":
    main()
