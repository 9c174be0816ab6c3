#!/usr/bin/env python3
"""tools/ab_libs.py -- A/B two builds of libspmm_hip.so (same C ABI) on the same HBM-resident A, B, C.

  python tools/ab_libs.py --lib lib_a.so --lib lib_b.so [...] --gen "<line>" --k 8
Interleaves the two handles over --rounds rounds (HIP events on the launch stream) and checks that the outputs agree.
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", required=True, help="library paths (the first is the reference)")
    ap.add_argument("--gen", action="append", required=True)
    ap.add_argument("--k", default="32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    libs = {Path(p).name: S._bind_hip(C.CDLL(p, mode=C.RTLD_LOCAL)) for p in args.lib}
    names = list(libs)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    for gen in args.gen:
        A = S.generate(S.gen_params(gen))
        for k in [int(x) for x in args.k.split(",")]:
            g = torch.Generator(device=dev)
            g.manual_seed(42)
            B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
            outs, hs, res = {}, {}, {n: [] for n in names}
            for n, L in libs.items():
                h = C.c_void_p()
                st = L.spmm_hip_create(A.row_ptr, A.col_idx, A.values.ctypes.data_as(C.c_void_p), A.m, A.ncols,
                                       A.nnz, k, S.F64, 0, C.byref(h))
                assert st == 0, st
                hs[n] = h
                outs[n] = torch.empty((A.m, k), device=dev, dtype=torch.float64)
            for _ in range(args.rounds):
                for n, L in libs.items():
                    run = lambda: L.spmm_hip_run_device(hs[n], C.c_void_p(B.data_ptr()), S.B_ROW_MAJOR,  # noqa
                                                        C.c_void_p(outs[n].data_ptr()), k, sp)
                    run()
                    run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        run()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    res[n].append(e0.elapsed_time(e1) / args.iters)
            close = all(bool(torch.allclose(outs[names[0]], outs[n], rtol=1e-12, atol=0)) for n in names)
            print(json.dumps({"gen": gen, "k": k, "ms": {n: float(np.median(res[n])) for n in names},
                              "close": close}), flush=True)
            for n, L in libs.items():
                L.spmm_hip_destroy(hs[n])


if __name__ == "__main__":
    main()
