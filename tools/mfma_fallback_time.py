#!/usr/bin/env python3
"""tools/mfma_fallback_time.py -- the cost of the matrix-core tiles' exact fallback: per line and K, a
launch with an in-range B, with one NaN in B and with one subnormal in B (each takes mfma_fixup_kernel's sparse
recompute of every tile), and with the matrix-core tiles off (SPMM_HIP_MFMA=-1) for scale.  Prints one JSON line per
(line, K): ms of each case and whether the fallback launches matched the plan without matrix-core tiles on every
row both report exact.

  python tools/mfma_fallback_time.py --k 32,128
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
LINES = "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;" \
        "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", default=LINES)
    ap.add_argument("--k", default="32")
    ap.add_argument("--launches", type=int, default=10)
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)

    def timed(mf, B, C):
        for _ in range(2):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), B.shape[1], st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.launches):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), B.shape[1], st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.launches

    for line in args.lines.split(";"):
        A = S.generate(S.gen_params(line))
        for k in (int(x) for x in args.k.split(",")):
            g = torch.Generator(device=dev).manual_seed(7)
            B = torch.rand((A.ncols, k), device=dev, dtype=torch.float64, generator=g)
            cases = {"in_range": B}
            Bn = B.clone()
            Bn[A.ncols // 2, k // 2] = float("nan")
            cases["one_nan"] = Bn
            Bs = B.clone()
            Bs[A.ncols // 3, 1] = 2.0 ** -1060
            cases["one_subnormal"] = Bs
            rec = {"gen": line, "k": k}
            os.environ["SPMM_HIP_MFMA"] = "-1"
            off = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
            os.environ.pop("SPMM_HIP_MFMA")
            on = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
            rec["mode"] = on.tile_info()["mode"]
            ex = torch.from_numpy(on.exact_rows().astype(bool) & off.exact_rows().astype(bool)).to(dev)
            for name, Bc in cases.items():
                C1 = torch.empty((A.m, k), device=dev, dtype=torch.float64)
                C0 = torch.empty_like(C1)
                rec[f"ms_{name}"] = round(timed(on, Bc, C1), 5)
                rec[f"ms_off_{name}"] = round(timed(off, Bc, C0), 5)
                a, b = C1[ex], C0[ex]
                same = (a.view(torch.int64) == b.view(torch.int64)) | (torch.isnan(a) & torch.isnan(b))
                rec[f"bitexact_{name}"] = bool(same.all().item())
            on.close()
            off.close()
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
