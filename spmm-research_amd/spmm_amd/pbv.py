"""The perfect-balance K = 1 format (include/spmm_pbv.h, lib/libspmm_pbv.so), mirrored like ``MatrixFormat``.

The GPU form of the reference's "Custom_CSR_PBV" build (spmv_kernel_csr.cpp:68-80, :626-680): m row ends and nnz
nonzeros merged into one item sequence, 256 x E items per workgroup, E per lane.  Rows whose items sit in one lane are
the reference's serial bits (``exact_rows``); the others are lane / block pieces added in a fixed order.  No CPU
fallback: importing this module without the built library raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import F32, F64, SpmmHipError, _i32p, _open

E_CHOICES = (4, 8, 16)
INFO = ("blocks", "items_per_lane", "exact_rows", "block_cut_rows", "device_bytes")


def _bind(L: C.CDLL) -> C.CDLL:
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.spmm_pbv_nblk.argtypes = [i64, i64, i32]
    L.spmm_pbv_nblk.restype = i64
    L.spmm_pbv_plan_host.argtypes = [_i32p, i64, i64, i32, vp, vp]
    L.spmm_pbv_create.argtypes = [_i32p, _i32p, vp, i64, i64, i64, i32, i32, i32, C.POINTER(vp)]
    L.spmm_pbv_run.argtypes = [vp, vp, vp, i32]
    L.spmm_pbv_run_device.argtypes = [vp, vp, vp, i64, vp]
    L.spmm_pbv_last_ms.argtypes = [vp, C.POINTER(C.c_double)]
    L.spmm_pbv_exact_rows.argtypes = [vp, vp]
    L.spmm_pbv_info.argtypes = [vp, C.POINTER(i64), i32]
    L.spmm_pbv_stats_labels.argtypes = [C.c_char_p, C.c_long]
    L.spmm_pbv_stats.argtypes = [vp, C.c_char_p, C.c_long]
    L.spmm_pbv_destroy.argtypes = [vp]
    L.spmm_pbv_last_error_detail.restype = C.c_char_p
    return L


lib = _bind(_open("libspmm_pbv.so"))


def _check(where: str, st: int):
    if st != 0:
        d = lib.spmm_pbv_last_error_detail()
        raise SpmmHipError(where, st, d.decode() if d else "")


def plan_host(row_ptr: np.ndarray, m: int, nnz: int, items_per_lane: int = 8) -> tuple[np.ndarray, np.ndarray]:
    """Host-only plan: (block starts int32 [nblk+1, 2] = {row, nonzero}, exact-row mask bool [m])."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    nblk = int(lib.spmm_pbv_nblk(m, nnz, items_per_lane))
    blk = np.zeros((nblk + 1, 2), np.int32)
    ex = np.zeros(max(m, 1), np.uint8)
    _check("plan_host", lib.spmm_pbv_plan_host(rp, m, nnz, items_per_lane, blk.ctypes.data_as(C.c_void_p),
                                               ex.ctypes.data_as(C.c_void_p)))
    return blk, ex[:m].astype(bool)


class PBVFormat:
    """``struct Matrix_Format`` of the PBV build (spmv_kernel.h:9-26) on one GPU; spmm(x, y, k) runs k SpMVs."""

    format_name = "HIP_CSR_PBV_MI355X"

    def __init__(self, row_ptr, col_ind, values, m: int, n: int, nnz: int, device: int = 0, items_per_lane: int = 8):
        self.m, self.n, self.nnz = int(m), int(n), int(nnz)
        vals = np.ascontiguousarray(values)
        if vals.dtype not in (np.float64, np.float32):
            raise TypeError("values must be float64 or float32 (ValueType)")
        self.dtype = np.dtype(vals.dtype)
        self._dt = F64 if self.dtype == np.float64 else F32
        rp = np.ascontiguousarray(row_ptr, np.int32)
        ci = np.ascontiguousarray(col_ind, np.int32)
        if len(ci) == 0:
            ci, vals = np.zeros(1, np.int32), np.zeros(1, self.dtype)
        self._h = C.c_void_p()
        _check("csr_to_format", lib.spmm_pbv_create(rp, ci, vals.ctypes.data_as(C.c_void_p), self.m, self.n, self.nnz,
                                                    self._dt, int(device), int(items_per_lane), C.byref(self._h)))

    def spmm(self, x: np.ndarray, y: np.ndarray, k: int = 1) -> None:
        """Host x column-major [k][n], host y row-major [m][k] (overwritten); synchronous."""
        if x.dtype != self.dtype or y.dtype != self.dtype:
            raise TypeError("x and y must have the handle's ValueType")
        if x.size < self.n * k or y.size < self.m * k or not (x.flags.c_contiguous and y.flags.c_contiguous):
            raise ValueError("x must hold n*k and y m*k contiguous values")
        _check("spmm", lib.spmm_pbv_run(self._h, x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), k))

    def spmv_device(self, d_x: int, d_y: int, ldy: int = 1, stream: int = 0) -> None:
        _check("spmv_device", lib.spmm_pbv_run_device(self._h, C.c_void_p(d_x), C.c_void_p(d_y), ldy,
                                                      C.c_void_p(stream)))

    def last_ms(self) -> float:
        t = C.c_double()
        _check("last_ms", lib.spmm_pbv_last_ms(self._h, C.byref(t)))
        return t.value

    def exact_rows(self) -> np.ndarray:
        out = np.zeros(max(self.m, 1), np.uint8)
        _check("exact_rows", lib.spmm_pbv_exact_rows(self._h, out.ctypes.data_as(C.c_void_p)))
        return out[:self.m].astype(bool)

    def info(self) -> dict:
        out = (C.c_int64 * len(INFO))()
        _check("info", lib.spmm_pbv_info(self._h, out, len(INFO)))
        return dict(zip(INFO, (int(v) for v in out)))

    def statistics_print_data(self) -> str:
        buf = C.create_string_buffer(512)
        n = lib.spmm_pbv_stats(self._h, buf, 512)
        if n < 0:
            _check("stats", n)
        return buf.value.decode()

    def close(self) -> None:
        if self._h:
            lib.spmm_pbv_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def statistics_print_labels() -> str:
    buf = C.create_string_buffer(512)
    lib.spmm_pbv_stats_labels(buf, 512)
    return buf.value.decode()
