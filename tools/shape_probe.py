#!/usr/bin/env python3
"""tools/shape_probe.py -- where the row kernel's time goes on dense-row lines (verdict r05 item 1).

For each generator line (K = 32 fp64, B rows of 256 B): the engine's own launch (its plan, as shipped, and with the
matrix-core tiles off), then the probes of tools/shape_probe.hip on the same column stream and the same B:
  flat        the column stream gathered by all 16 row groups of every workgroup (no row structure, full occupancy);
  rows_gather the kernel's block structure (<= 2048 nonzeros staged per workgroup, one row per 16-lane group, U = 16
              gathers in flight, one C row stored per row), B rows summed (no A values);
  rows_fma    the same with the A values staged and an FMA chain per row (the row kernel's arithmetic);
  rows_fma_8k the same with 8,192 nonzeros per workgroup (all four waves busy on 500-nonzero rows).
Each prints one JSON line: ms per launch and the B-row rate (nnz x 256 B / time).  Run it under rocprofv3 --pmc to
get the counters of each kernel (the kernel names tell them apart).

  python tools/shape_probe.py --lines "5588 5588 500 166.6667 normal random 0.3 1000 1.9 0.5 14;..."
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def blocks(rp: np.ndarray, cap: int, piece: int = 2048, max_pieces: int = 512):
    """Rows cut into pieces of <= `piece` nonzeros, packed greedily into blocks of <= cap nonzeros (and <=
    max_pieces pieces): (block -> first piece [nblk+1], piece offsets [np+1])."""
    starts = []
    for i in range(len(rp) - 1):
        a, e = int(rp[i]), int(rp[i + 1])
        if e == a:
            continue
        for s in range(a, e, piece):
            starts.append(s)
    pp = np.array(starts + [int(rp[-1])], np.int32)
    blk = [0]
    n = 0
    cnt = 0
    for p in range(len(pp) - 1):
        ln = int(pp[p + 1] - pp[p])
        if cnt and (n + ln > cap or cnt >= max_pieces):
            blk.append(p)
            n, cnt = 0, 0
        n += ln
        cnt += 1
    blk.append(len(pp) - 1)
    return np.array(blk, np.int32), pp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", required=True, help="generator lines separated by ';'")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    L = C.CDLL(str(ROOT / "spmm-research_amd" / "lib" / "libshape_probe.so"))
    L.probe_flat.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    L.probe_rows.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                             C.c_void_p, C.c_void_p]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    K = 32

    def timeit(fn, iters):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    for line in [x.strip() for x in args.lines.split(";") if x.strip()]:
        A = S.generate(S.gen_params(line))
        g = torch.Generator(device=dev)
        g.manual_seed(42)
        B = torch.rand((A.ncols, K), generator=g, device=dev, dtype=torch.float64)
        Cd = torch.empty((A.m, K), device=dev, dtype=torch.float64)
        bytes_b = A.nnz * K * 8
        rec = {"gen": line, "m": A.m, "nnz": A.nnz, "b_mb": A.ncols * K * 8 / 2 ** 20}
        for name, env in (("engine", {}), ("engine_rows", {"SPMM_HIP_MFMA": "-1", "SPMM_HIP_TILES": "-1"})):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, K, 0)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            ms = timeit(lambda: mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), K, st.cuda_stream),
                        args.iters)
            rec[name] = {"ms": round(ms, 5), "b_rows_tbs": round(bytes_b / (ms * 1e-3) / 1e12, 2),
                         "tiles": int(mf.info()[19]), "split_rows": int(mf.info()[6])}
            mf.close()
        col = torch.from_numpy(A.col_idx).to(dev)
        val = torch.from_numpy(A.values).to(dev)
        out = torch.empty(((A.nnz + 2047) // 2048) * 256 * 2, device=dev, dtype=torch.float64)
        ms = timeit(lambda: L.probe_flat(C.c_void_p(col.data_ptr()), A.nnz, C.c_void_p(B.data_ptr()),
                                         C.c_void_p(out.data_ptr()), sp), args.iters)
        rec["flat"] = {"ms": round(ms, 5), "b_rows_tbs": round(bytes_b / (ms * 1e-3) / 1e12, 2)}
        for var, name, cap in ((0, "rows_gather", 2048), (1, "rows_fma", 2048), (2, "rows_fma_8k", 8192)):
            blk, pp = blocks(A.row_ptr, cap)
            dblk = torch.from_numpy(blk).to(dev)
            dpp = torch.from_numpy(pp).to(dev)
            Cp = torch.empty((len(pp) * K,), device=dev, dtype=torch.float64)
            nb = len(blk) - 1
            ms = timeit(lambda: L.probe_rows(var, C.c_void_p(dblk.data_ptr()), nb, C.c_void_p(dpp.data_ptr()),
                                             C.c_void_p(col.data_ptr()), C.c_void_p(val.data_ptr()),
                                             C.c_void_p(B.data_ptr()), C.c_void_p(Cp.data_ptr()), sp), args.iters)
            rec[name] = {"ms": round(ms, 5), "b_rows_tbs": round(bytes_b / (ms * 1e-3) / 1e12, 2), "blocks": nb,
                         "pieces": len(pp) - 1}
            del dblk, dpp, Cp
        print(json.dumps(rec), flush=True)
        del A, B, Cd, col, val, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
