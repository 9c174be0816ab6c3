#!/usr/bin/env python3
"""tools/pbv_ab.py -- K = 1: the perfect-balance format (include/spmm_pbv.h, E items per lane) against the engine's
row kernel (include/spmm_hip.h) on the same matrices, same x, one process, HIP events.

Lines: --per-class N lines of every (avg nnz/row, bw) class of the medium dataset (evenly spaced, <= --max-nnz), plus
config 2 (1M x 1M, 20/row).  Per line and format: the lowest of 3 batch means of --iters launches after --warmup, the
exact-row fraction, and a bit-equality check of the rows both formats report exact.  One JSON line per matrix.

  python tools/pbv_ab.py --per-class 3 --out gpurun_out/pbv/ab.jsonl
"""
import argparse
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
sys.path.insert(0, str(ROOT))
CONFIG2 = "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"


def lines(per_class, max_nnz):
    from spmm_amd.datasets import medium_dataset_lines
    cls = defaultdict(list)
    for line in medium_dataset_lines():
        g = line.split()
        if int(g[0]) * float(g[2]) <= max_nnz:
            cls[(int(g[2]), float(g[6]))].append(line)
    out = []
    for key in sorted(cls):
        c = cls[key]
        out += [c[i] for i in sorted(set(np.linspace(0, len(c) - 1, per_class).round().astype(int)))]
    return [CONFIG2] + out


def timed(torch, stream, run, warmup, iters):
    for _ in range(warmup):
        run()
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            run()
        e1.record(stream)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-class", type=int, default=3)
    ap.add_argument("--max-nnz", type=float, default=6e7)
    ap.add_argument("--e", default="4,8,16")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--budget", type=float, default=900)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "pbv" / "ab.jsonl"))
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    import spmm_amd.pbv as P
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    out = Path(args.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    t0 = time.time()
    es = [int(e) for e in args.e.split(",")]
    for line in lines(args.per_class, args.max_nnz):
        if time.time() - t0 > args.budget:
            print("budget reached", flush=True)
            break
        A = S.generate(S.gen_params(line))
        g = torch.Generator(device=dev)
        g.manual_seed(42)
        x = torch.rand((max(A.ncols, 1), 1), generator=g, device=dev, dtype=torch.float64)
        y0 = torch.empty((max(A.m, 1), 1), device=dev, dtype=torch.float64)
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, 1, 0)
        ms_row = timed(torch, stream, lambda: mf.spmm_device(x.data_ptr(), S.B_ROW_MAJOR, y0.data_ptr(), 1,
                                                               stream.cuda_stream), args.warmup, args.iters)
        ex0 = mf.exact_rows()
        mf.close()
        rec = {"gen": line, "m": A.m, "nnz": A.nnz, "ms_row": ms_row, "exact_row": float(ex0.mean()),
               "bytes_alg": S.bytes_alg(A.m, A.ncols, A.nnz, 1, S.F64)}
        Y0 = y0.cpu().numpy().ravel()
        for e in es:
            f = P.PBVFormat(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, 0, e)
            y1 = torch.empty_like(y0)
            ms = timed(torch, stream, lambda: f.spmv_device(x.data_ptr(), y1.data_ptr(), 1, stream.cuda_stream),
                       args.warmup, args.iters)
            ex1 = f.exact_rows()
            Y1 = y1.cpu().numpy().ravel()
            both = ex0 & ex1
            rec[f"ms_pbv{e}"] = ms
            rec[f"exact_pbv{e}"] = float(ex1.mean())
            rec[f"bitequal_pbv{e}"] = bool(np.array_equal(Y0[both].view(np.int64), Y1[both].view(np.int64)))
            rec[f"speedup_pbv{e}"] = ms_row / ms
            f.close()
        with open(out, "a") as fh:
            fh.write(json.dumps(rec) + "\n")
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items() if k != "gen"}),
              flush=True)
        del A, x, y0


if __name__ == "__main__":
    main()
