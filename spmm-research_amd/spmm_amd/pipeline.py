"""spmm_amd.pipeline -- the sparse-attention pipeline consumer on the engine.

Mirror of the reference's pipeline bench (benchmark_code/CPU/AMD/pipeline_code_bench/sddmm_bench.cpp, compute()
:531-990 with the default branch :918-937, and its plugin surface sddmm_kernel.h:9-31):

    K = W_K x,  Q = W_Q x,  V = W_V x           MF->spmm('K'|'Q'|'V', m, k, n, ia, ja, a, x, y)   (row-major x, y)
    y = SDDMM(mask, Q, K)                        MF->sddmm(y)            (sddmm_taco_naive.cpp:98-140, 211-217)
    y_final = mask(y) V                          MF->spmm('final', m, m, n, mask ia, mask ja, y, V, y_final)

GFLOP/s as the reference reports it (sddmm_bench.cpp:978-983): 2 n (nnz_K + nnz_Q + nnz_V + 2 nnz_mask) / time.
The SpMMs run on the engine (C ABI, spmm_hip.h) with B row-major; the SDDMM (and the optional softmax the
reference has commented out) on spmm_sddmm (spmm_pipeline.h); the final SpMM takes the SDDMM output as its
values on the device (spmm_hip_update_values_device).  Everything is stream-ordered, so one pipeline step can
be captured in a hipGraph.

Inputs (the reference reads three DLMC .smtx transformer weights and builds the mask with time-seeded rand(),
sddmm_mask.h:16-80 -- neither is reproducible offline): ``dlmc_like_weight`` draws a seeded uniform-random
pruned m x k weight (U[-1,1) values, like smtx_read's values), ``band_and_random_mask`` restates the reference's
band + random-lower-triangle mask with a seeded generator, values 1.0.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import CSR, F32, F64, B_ROW_MAJOR, SpmmHipError, csr_to_format, hip, run_device_batch

SDDMM_REF_ROWDIAG, SDDMM_QKT, SDDMM_SOFTMAX = 0, 1, 2


def dlmc_like_weight(m: int, k: int, density: float, seed: int) -> CSR:
    """A pruned transformer weight like the DLMC ones (random pruning): each entry kept with probability
    `density`, values U[-1, 1), columns sorted, seeded."""
    rng = np.random.default_rng(seed)
    keep = rng.random((m, k)) < density
    rows, cols = np.nonzero(keep)
    row_ptr = np.zeros(m + 1, np.int32)
    np.cumsum(np.bincount(rows, minlength=m), out=row_ptr[1:])
    vals = rng.uniform(-1.0, 1.0, len(cols))
    return CSR(row_ptr, cols.astype(np.int32), vals, m, k)


def band_and_random_mask(m: int, density: float, band_size: int, seed: int) -> CSR:
    """sddmm_mask.h:16-80 (band_and_random) restated with a seeded generator: every (i, j) with |i-j| < band_size,
    then uniformly random lower-triangle (j <= i) entries until round(density * m*m) nonzeros (or the lower
    triangle is full); row-major CSR with sorted columns (dense_to_csr, :272-294), values 1.0."""
    mask = np.zeros((m, m), bool)
    ii = np.arange(m)
    for d in range(-(band_size - 1), band_size):
        j = ii + d
        ok = (j >= 0) & (j < m)
        mask[ii[ok], j[ok]] = True
    target = int(density * m * m)
    lower = np.tril(np.ones((m, m), bool))
    free = np.flatnonzero(lower & ~mask)
    need = max(0, min(target - int(mask.sum()), len(free)))
    if need:
        rng = np.random.default_rng(seed)
        mask.flat[rng.choice(free, need, replace=False)] = True
    rows, cols = np.nonzero(mask)
    row_ptr = np.zeros(m + 1, np.int32)
    np.cumsum(np.bincount(rows, minlength=m), out=row_ptr[1:])
    return CSR(row_ptr, cols.astype(np.int32), np.ones(len(cols)), m, m)


class Sddmm:
    """Handle of the engine's SDDMM (spmm_sddmm_*): the mask's SDDMM with Q, K ([rows][n] row-major)."""

    def __init__(self, mask: CSR, n: int, dtype=np.float64, flags: int = SDDMM_REF_ROWDIAG, device: int = 0):
        self.dtype = np.dtype(dtype)
        self.m, self.nnz, self.n, self.flags = mask.m, mask.nnz, int(n), int(flags)
        vals = np.ascontiguousarray(mask.values, self.dtype)
        ci = mask.col_idx if len(mask.col_idx) else np.zeros(1, np.int32)
        if len(vals) == 0:
            vals = np.zeros(1, self.dtype)
        self._h = C.c_void_p()
        st = hip.spmm_sddmm_create(np.ascontiguousarray(mask.row_ptr, np.int32), np.ascontiguousarray(ci, np.int32),
                                   vals.ctypes.data_as(C.c_void_p), mask.m, mask.ncols, mask.nnz, self.n,
                                   F64 if self.dtype == np.float64 else F32, self.flags, device, C.byref(self._h))
        if st != 0:
            raise SpmmHipError("sddmm_create", st, (hip.spmm_sddmm_last_error_detail() or b"").decode())

    def run(self, Q: np.ndarray, K: np.ndarray) -> np.ndarray:
        Q = np.ascontiguousarray(Q, self.dtype)
        K = np.ascontiguousarray(K, self.dtype)
        y = np.empty(max(self.nnz, 1), self.dtype)
        st = hip.spmm_sddmm_run(self._h, Q.ctypes.data_as(C.c_void_p), K.ctypes.data_as(C.c_void_p), K.shape[0],
                                y.ctypes.data_as(C.c_void_p))
        if st != 0:
            raise SpmmHipError("sddmm_run", st, (hip.spmm_sddmm_last_error_detail() or b"").decode())
        return y[:self.nnz]

    def run_device(self, d_q: int, d_k: int, d_y: int, stream: int = 0) -> None:
        st = hip.spmm_sddmm_run_device(self._h, C.c_void_p(d_q), C.c_void_p(d_k), C.c_void_p(d_y),
                                       C.c_void_p(stream))
        if st != 0:
            raise SpmmHipError("sddmm_run_device", st, (hip.spmm_sddmm_last_error_detail() or b"").decode())

    def close(self) -> None:
        if self._h:
            hip.spmm_sddmm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SparseAttentionPipeline:
    """K/Q/V SpMMs, SDDMM (+ optional softmax), final SpMM -- the reference compute() step (sddmm_bench.cpp:918-937)."""

    def __init__(self, w_k: CSR, w_q: CSR, w_v: CSR, mask: CSR, n: int, dtype=np.float32,
                 sddmm_flags: int = SDDMM_REF_ROWDIAG, device: int = 0):
        if not (w_k.ncols == w_q.ncols == w_v.ncols):
            raise ValueError("W_K, W_Q, W_V must share their column count (x has k rows)")
        if mask.m != w_q.m or mask.m != w_v.m or (sddmm_flags & 1 and mask.ncols > w_k.m) or \
                (not sddmm_flags & 1 and mask.m > w_k.m):
            raise ValueError("mask rows must match W_Q / W_V rows and fit W_K (the reference uses m = rows of W_K)")
        self.dtype = np.dtype(dtype)
        self.n = int(n)
        self.w = {"K": w_k, "Q": w_q, "V": w_v}
        self.mask = mask
        self.mf = {t: csr_to_format(a.row_ptr, a.col_idx, a.values.astype(self.dtype), a.m, a.ncols, a.nnz, self.n,
                                    device) for t, a in self.w.items()}
        self.final = csr_to_format(mask.row_ptr, mask.col_idx, mask.values.astype(self.dtype), mask.m, mask.ncols,
                                   mask.nnz, self.n, device)
        self.sddmm = Sddmm(mask, self.n, self.dtype, sddmm_flags, device)
        self.flops = 2.0 * self.n * (w_k.nnz + w_q.nnz + w_v.nnz + 2 * mask.nnz)

    def run_device(self, d_x: int, d_k: int, d_q: int, d_v: int, d_y: int, d_out: int, stream: int = 0) -> None:
        """One pipeline step on device buffers (row-major): x [k][n] -> K, Q, V [m][n], y [mask nnz], out [m][n]."""
        # the three projections are independent: one concurrent batch (side streams forked from `stream`)
        run_device_batch([(self.mf[t], d_x, B_ROW_MAJOR, d, self.n) for t, d in (("K", d_k), ("Q", d_q), ("V", d_v))],
                         stream)
        self.sddmm.run_device(d_q, d_k, d_y, stream)
        self.final.update_values_device(d_y, stream)
        self.final.spmm_device(d_v, B_ROW_MAJOR, d_out, self.n, stream)

    def run(self, x: np.ndarray) -> dict:
        """Host path with the reference plugin's call sequence: returns K, Q, V, y (mask values), y_final."""
        x = np.ascontiguousarray(x, self.dtype)
        out = {}
        for t in ("K", "Q", "V"):
            y = np.empty(self.w[t].m * self.n, self.dtype)
            self.mf[t].spmm_rowmajor(x, y, self.n)
            out[t] = y.reshape(self.w[t].m, self.n)
        out["y"] = self.sddmm.run(out["Q"], out["K"])
        self.final.update_values(out["y"])
        yf = np.empty(self.mask.m * self.n, self.dtype)
        self.final.spmm_rowmajor(np.ascontiguousarray(out["V"]), yf, self.n)
        out["y_final"] = yf.reshape(self.mask.m, self.n)
        return out

    def close(self) -> None:
        for mf in list(self.mf.values()) + [self.final]:
            mf.close()
        self.sddmm.close()
