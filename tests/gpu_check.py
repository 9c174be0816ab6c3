"""Shared GPU-test helpers: run a matrix through the engine (C ABI, HBM-resident) and check a row sample against the
oracle (tests only).

Parity contract: rows the engine reports exact (spmm_hip_exact_rows) must be BIT-IDENTICAL to the oracle's
restatement of compute_csr (benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:70-96); every sampled row
must be within 1e-10 normwise of the __float128 gold (fp64) or (n+1)*2^-24 (fp32 sequential sums).
"""
from __future__ import annotations

import numpy as np


def run_device(torch, S, A, k, dtype=np.float64, seed=9, device=0):
    """B = seeded U[0,1) row-major in HBM, C row-major; returns (B host, C host, info, exact mask)."""
    dev = torch.device("cuda", device)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    B = torch.rand((max(A.ncols, 1), k), generator=g, device=dev, dtype=tdt)
    C = torch.full((max(A.m, 1), k), float("nan"), device=dev, dtype=tdt)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(dtype), A.m, A.ncols, A.nnz, k, device)
    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    inf, ex = mf.info(), mf.exact_rows()
    mf.close()
    return B.cpu().numpy(), C.cpu().numpy()[:A.m], inf, ex


def check_rows(O, A, B, C, ex, rows, dtype=np.float64):
    """Oracle on the given rows (sub-CSR with renumbered columns): exact rows bit for bit, all rows normwise.
    Returns (number of exact rows checked, number of inexact rows checked)."""
    rows = np.asarray(rows, np.int64)
    deg = np.diff(A.row_ptr)[rows]
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    if rp[-1] > 0:
        cols = np.concatenate([A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows])
        vals = np.concatenate([A.values[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows])
    else:
        cols, vals = np.zeros(0, np.int32), np.zeros(0)
    uc, inv = np.unique(cols, return_inverse=True)
    k = B.shape[1]
    x = np.ascontiguousarray(B[uc].T).reshape(-1)
    vv = vals.astype(dtype)
    want = O.spmm(rp, inv.astype(np.int32), vv, max(len(uc), 1), x.astype(dtype) if len(x) else np.zeros(k, dtype), k)
    got = C[rows]
    exr = ex[rows].astype(bool)
    it = np.int64 if dtype == np.float64 else np.int32
    assert np.array_equal(got[exr].view(it), want[exr].view(it)), "exact rows differ from the oracle"
    g, absdot = O.gold(rp, inv.astype(np.int32), vv.astype(np.float64), max(len(uc), 1),
                       x.astype(np.float64) if len(x) else np.zeros(k), k)
    if dtype == np.float64:
        ok = O.normwise_ok(got, g, absdot, 1e-10)
    else:
        tol = (np.maximum(deg, 1)[:, None] + 1) * 2.0 ** -24 * 1.01
        ok = np.abs(got.astype(np.float64) - g) <= tol * np.maximum(np.abs(g), absdot)
    assert ok.all(), f"{int((~ok).sum())} entries outside the normwise bound"
    return int(exr.sum()), int((~exr).sum())


def sample_rows(A, n=2000, seed=1, include_longest=True):
    rng = np.random.default_rng(seed)
    rows = rng.choice(A.m, min(n, A.m), replace=False) if A.m else np.zeros(0, np.int64)
    if include_longest and A.m:
        deg = np.diff(A.row_ptr)
        rows = np.concatenate([rows, np.argsort(deg)[-8:]])
    return np.unique(rows)
