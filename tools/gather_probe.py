#!/usr/bin/env python3
"""tools/gather_probe.py -- gather-rate ceilings on this GPU (measurement only; see tools/gather_probe.hip).

Prints one JSON line per case: 256-B row gathers/s and GB/s for random rows over tables sized for L2, the Infinity
Cache and HBM, for the benchmark matrix's own col_idx stream (gather-only: the SpMM kernel's B traffic without
A, C or row structure), plus a plain streaming read (HBM ceiling)."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    import torch
    import spmm_amd as S
    L = C.CDLL(str(ROOT / "spmm-research_amd" / "lib" / "libgather_probe.so"))
    L.probe_gather.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
    L.probe_fill_idx.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_uint64, C.c_void_p]
    L.probe_stream.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    n = 20_000_000
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    out = torch.empty(64 << 20, dtype=torch.float64, device=dev)

    def timeit(fn, iters=10):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e-3

    # random 256-B rows over tables of increasing size
    for mb in (2, 16, 64, 160, 256, 1024, 4096):
        rows = mb * (1 << 20) // 256
        table = torch.rand(rows * 32, dtype=torch.float64, device=dev)
        L.probe_fill_idx(C.c_void_p(idx.data_ptr()), n, rows, 1234, sp)
        for u, pg in ((16, 128), (8, 128)):
            t = timeit(lambda: L.probe_gather(C.c_void_p(idx.data_ptr()), n, C.c_void_p(table.data_ptr()),
                                              C.c_void_p(out.data_ptr()), pg, u, sp))
            print(json.dumps({"case": f"random_rows_table_{mb}MB", "U": u, "ms": t * 1e3,
                              "gather_TBps": n * 256 / t / 1e12}), flush=True)
        del table
    # the benchmark matrix's col_idx stream against its B
    A = S.generate(S.gen_params("1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"))
    ci = torch.from_numpy(A.col_idx).to(dev)
    table = torch.rand(A.ncols * 32, dtype=torch.float64, device=dev)
    for u, pg in ((16, 128), (8, 128)):
        t = timeit(lambda: L.probe_gather(C.c_void_p(ci.data_ptr()), A.nnz, C.c_void_p(table.data_ptr()),
                                          C.c_void_p(out.data_ptr()), pg, u, sp))
        print(json.dumps({"case": "config2_col_idx_stream", "U": u, "per_group": pg, "ms": t * 1e3,
                          "gather_TBps": A.nnz * 256 / t / 1e12}), flush=True)
    # streaming read ceiling (4 GiB)
    big = torch.empty(512 << 20, dtype=torch.float64, device=dev).fill_(1.0)
    t = timeit(lambda: L.probe_stream(C.c_void_p(big.data_ptr()), big.numel() // 2, C.c_void_p(out.data_ptr()),
                                      8192, sp))
    print(json.dumps({"case": "stream_read_4GiB", "ms": t * 1e3, "TBps": big.numel() * 8 / t / 1e12}), flush=True)


if __name__ == "__main__":
    main()
