#!/usr/bin/env python3
"""tools/mfma_ab.py -- A/B of the matrix-core tiles against the same engine with them off
(SPMM_HIP_MFMA=-1: exactly the plan of the engine before round 3's matrix-core tiles) on medium-dataset lines.

For each line x K: two handles on the same HBM-resident B (seeded uniform [-1, 1)), launches interleaved over rounds
(HIP events, lowest of --rounds batch means of --iters launches); rows exact in both plans must be bit-identical.
One JSON line per case: times, tile mode / rows / chunks of the policy plan, algorithmic-byte roofline fractions.

  python tools/mfma_ab.py --stride 160 --min-avg 20 --k 32,128 > ab.jsonl
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", default="", help="';'-separated generator lines (default: a dataset sample)")
    ap.add_argument("--stride", type=int, default=160)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--min-avg", type=float, default=0.0, help="only lines with at least this many nonzeros per row")
    ap.add_argument("--max-nnz", type=float, default=1.6e8)
    ap.add_argument("--k", default="32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--budget", type=float, default=1e9, help="seconds; no new line after this")
    ap.add_argument("--modes", default="off:SPMM_HIP_MFMA=-1;on:",
                    help="';'-separated name:ENV=V,ENV=V handles to compare (the first is the baseline)")
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    from spmm_amd.datasets import medium_dataset_lines
    if args.lines:
        lines = args.lines.split(";")
    else:
        lines = [l for l in medium_dataset_lines()[args.offset::args.stride] if float(l.split()[2]) >= args.min_avg]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    t0 = time.time()
    for line in lines:
        if time.time() - t0 > args.budget:
            break
        p = S.gen_params(line)
        A = S.generate(p)
        if A.nnz > args.max_nnz:
            continue
        for k in (int(x) for x in args.k.split(",")):
            g = torch.Generator(device=dev)
            g.manual_seed(42)
            B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64) * 2 - 1
            hs = {}
            modes = []
            for spec in args.modes.split(";"):
                name, _, kv = spec.partition(":")
                modes.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
            for name, env in modes:
                for kk, vv in env.items():
                    os.environ[kk] = vv
                hs[name] = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
                for kk in env:
                    os.environ.pop(kk)
            Cs = {n: torch.empty((A.m, k), device=dev, dtype=torch.float64) for n in hs}
            ts = {n: [] for n in hs}
            for _ in range(args.rounds):
                for n, h in hs.items():
                    h.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cs[n].data_ptr(), k, sp)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        h.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cs[n].data_ptr(), k, sp)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ts[n].append(e0.elapsed_time(e1) / args.iters)
            n0, n1 = modes[0][0], modes[-1][0]
            exm = hs[n0].exact_rows()
            for h_ in hs.values():
                exm = exm & h_.exact_rows()
            ex = torch.from_numpy(exm).to(dev)
            same = all(bool(torch.equal(Cs[n][ex].view(torch.int64), Cs[n0][ex].view(torch.int64))) for n in hs)
            ti = hs[n1].tile_info()
            ba = S.bytes_alg(A.m, A.ncols, A.nnz, k, S.F64)
            t_off, t_on = min(ts[n0]), min(ts[n1])
            rec = {"gen": line, "k": k, "m": A.m, "nnz": A.nnz, "off_ms": round(t_off, 5), "on_ms": round(t_on, 5),
                   "speedup": round(t_off / t_on, 3), "mode": ti["mode"], "tile_rows": ti["rows"],
                   "tile_nnz": ti["nnz"], "chunks": ti["chunks"], "reuse": ti["reuse"],
                   "frac_off": round(ba / (t_off * 1e-3) / 8e12, 4), "frac_on": round(ba / (t_on * 1e-3) / 8e12, 4),
                   "gflops_on": round(2.0 * A.nnz * k / t_on / 1e6, 1), "exact_rows_both": int(ex.sum().item()),
                   "bitexact": same, "ms": {n: round(min(ts[n]), 5) for n in ts}}
            print(json.dumps(rec), flush=True)
            for h in hs.values():
                h.close()
            del B, Cs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
