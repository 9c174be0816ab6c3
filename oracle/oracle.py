"""oracle/oracle.py -- ctypes access to the CPU checker libraries.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
the product (spmm-research_amd/).  Two libraries:

* ``liboracle.so``  -- our C restatement of the reference hot path (oracle/spmm_oracle.c; each function cites the
  reference file:line it restates).
* ``_ref/libspmm_ref_{d,f}.so`` -- the reference's own sources compiled by oracle/Makefile (optional: present when
  built in the container that has /root/reference, and shipped prebuilt to the GPU box).

Parity of the restatement is pinned by tests/test_oracle_golden.py against fixtures the reference produced
(tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


def _load(name: str) -> C.CDLL:
    path = HERE / name
    if not path.exists():
        raise FileNotFoundError(f"{path} not built (run `make -C oracle`)")
    return C.CDLL(str(path))


_oracle = None
_ref: dict[str, C.CDLL] = {}


def lib() -> C.CDLL:
    global _oracle
    if _oracle is None:
        L = _load("liboracle.so")
        i64 = C.c_int64
        L.oracle_spmm_csr_d.argtypes = [_i32p, _i32p, _f64p, i64, i64, _f64p, _f64p, C.c_int32, C.c_int32]
        L.oracle_spmm_csr_f.argtypes = [_i32p, _i32p, _f32p, i64, i64, _f32p, _f32p, C.c_int32, C.c_int32]
        L.oracle_binary_search.argtypes = [_i32p, i64, i64, i64]
        L.oracle_binary_search.restype = i64
        L.oracle_partition.argtypes = [_i32p, i64, i64, i64, i64, C.POINTER(i64), C.POINTER(i64)]
        L.oracle_gold_to_double.argtypes = [_i32p, _i32p, _f64p, i64, i64, _f64p, C.c_int32, _f64p, C.c_void_p]
        L.oracle_gold.argtypes = [_i32p, _i32p, _f64p, i64, i64, _f64p, C.c_int32, C.c_void_p]
        L.oracle_check_accuracy.argtypes = [C.c_void_p, _f64p, i64, C.c_double, _f64p]
        L.oracle_coo_to_csr.argtypes = [_i32p, _i32p, C.c_void_p, i64, i64, i64, _i32p, _i32p, _f64p]
        L.oracle_drand48_fill.argtypes = [i64, _f64p, i64]
        L.oracle_sddmm_d.argtypes = [_i32p, _i32p, _f64p, i64, _f64p, _f64p, C.c_int32, C.c_int32, _f64p]
        L.oracle_sddmm_f.argtypes = [_i32p, _i32p, _f32p, i64, _f32p, _f32p, C.c_int32, C.c_int32, _f32p]
        L.oracle_softmax_d.argtypes = [_f64p, i64]
        L.oracle_softmax_f.argtypes = [_f32p, i64]
        _oracle = L
    return _oracle


def ref_available(vt: str = "d") -> bool:
    return (HERE / "_ref" / f"libspmm_ref_{vt}.so").exists()


def ref_lib(vt: str = "d") -> C.CDLL:
    if vt not in _ref:
        L = _load(f"_ref/libspmm_ref_{vt}.so")
        vp = _f64p if vt == "d" else _f32p
        L.ref_spmm.argtypes = [_i32p, _i32p, vp, C.c_long, C.c_long, C.c_long, vp, vp, C.c_int]
        L.ref_create.argtypes = [_i32p, _i32p, vp, C.c_long, C.c_long, C.c_long, C.c_int]
        L.ref_create.restype = C.c_void_p
        L.ref_run.argtypes = [C.c_void_p, vp, vp, C.c_int]
        L.ref_destroy.argtypes = [C.c_void_p]
        L.ref_mtx_to_csr.argtypes = [C.c_char_p, C.POINTER(C.c_long), C.POINTER(C.c_long), C.POINTER(C.c_long),
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ref_free.argtypes = [C.c_void_p]
        L.ref_smtx_read.argtypes = [C.c_char_p, C.POINTER(C.c_long), C.POINTER(C.c_long), C.POINTER(C.c_long),
                                    C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.ref_partition.argtypes = [_i32p, C.c_long, C.c_long, C.c_long, C.c_long, C.POINTER(C.c_long),
                                    C.POINTER(C.c_long)]
        L.ref_metrics.argtypes = [_f64p, _f64p, C.c_long, _f64p]
        L.ref_set_threads.argtypes = [C.c_int]
        L.ref_features.argtypes = [_i32p, _i32p, C.c_long, C.c_long, C.c_long, C.c_char_p, C.c_long]
        L.ref_features.restype = C.c_long
        _ref[vt] = L
    return _ref[vt]


# ----------------------------------------------------------------------------------------------- restatement
def spmm(row_ptr, col_idx, vals, ncols: int, x_colmajor, k: int, nthreads: int = 0) -> np.ndarray:
    """compute_csr restated (spmm_kernel_csr.cpp:70-96): x column-major [k][ncols], returns y row-major [m][k]."""
    m = len(row_ptr) - 1
    if vals.dtype == np.float64:
        y = np.empty(m * k, np.float64)
        lib().oracle_spmm_csr_d(row_ptr, col_idx, vals, m, ncols, x_colmajor, y, k, nthreads)
    else:
        y = np.empty(m * k, np.float32)
        lib().oracle_spmm_csr_f(row_ptr, col_idx, vals, m, ncols, x_colmajor, y, k, nthreads)
    return y.reshape(m, k)


def partition(row_ptr, nnz: int, workers: int, pos: int) -> tuple[int, int]:
    s, e = C.c_int64(), C.c_int64()
    lib().oracle_partition(row_ptr, len(row_ptr) - 1, nnz, workers, pos, C.byref(s), C.byref(e))
    return s.value, e.value


def gold(row_ptr, col_idx, vals_ref, ncols: int, x_ref_colmajor, k: int):
    """CheckAccuracy gold (spmv_bench.cpp:130-160) rounded to double, plus sum_j |a_ij b_jn| per entry."""
    m = len(row_ptr) - 1
    g = np.empty(m * k, np.float64)
    ad = np.empty(m * k, np.float64)
    lib().oracle_gold_to_double(row_ptr, col_idx, vals_ref, m, ncols, x_ref_colmajor, k, g,
                                ad.ctypes.data_as(C.c_void_p))
    return g.reshape(m, k), ad.reshape(m, k)


def check_accuracy(row_ptr, col_idx, vals_ref, ncols: int, x_ref_colmajor, k: int, y_test, eps: float):
    """Full CheckAccuracy restatement: [maxreldiff, mae, max_ae, mse, mape, smape, lnQ, mlare, gmare]."""
    m = len(row_ptr) - 1
    N = m * k
    gold128 = (C.c_ubyte * (16 * max(N, 1)))()
    lib().oracle_gold(row_ptr, col_idx, vals_ref, m, ncols, x_ref_colmajor, k, C.cast(gold128, C.c_void_p))
    out = np.empty(9, np.float64)
    lib().oracle_check_accuracy(C.cast(gold128, C.c_void_p), np.ascontiguousarray(y_test, np.float64).ravel(),
                                N, eps, out)
    return out


def coo_to_csr(R, Cc, V, m: int, n: int | None = None):
    """coo_to_csr (csr_gen.c:163-217) as the reference runs it with one thread; n = column count (default
    max column + 1)."""
    nnz = len(R)
    Cc = np.ascontiguousarray(Cc, np.int32)
    ncols = (int(Cc.max()) + 1 if nnz else 0) if n is None else int(n)
    rp = np.empty(m + 1, np.int32)
    ci = np.empty(max(nnz, 1), np.int32)
    va = np.empty(max(nnz, 1), np.float64)
    vptr = None if V is None else np.ascontiguousarray(V, np.float64).ctypes.data_as(C.c_void_p)
    lib().oracle_coo_to_csr(np.ascontiguousarray(R, np.int32), Cc, vptr, m, ncols, nnz, rp, ci, va)
    return rp, ci[:nnz], va[:nnz]


def drand48(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, np.float64)
    lib().oracle_drand48_fill(seed, out, n)
    return out


def normwise_ok(y_test, y_gold, absdot, tol: float) -> np.ndarray:
    """|C_test - C_gold| <= tol * max(|C_gold|, sum_j |a_ij b_jn|) per entry."""
    bound = tol * np.maximum(np.abs(y_gold), absdot)
    return np.abs(np.asarray(y_test, np.float64) - y_gold) <= bound


# ------------------------------------------------------------------------------------------------ reference
def ref_spmm(row_ptr, col_idx, vals, ncols: int, x_colmajor, k: int) -> np.ndarray:
    vt = "d" if vals.dtype == np.float64 else "f"
    m = len(row_ptr) - 1
    y = np.zeros(m * k, vals.dtype)
    ref_lib(vt).ref_spmm(row_ptr, col_idx, vals, m, ncols, len(col_idx), x_colmajor, y, k)
    return y.reshape(m, k)


def ref_mtx_to_csr(path: str, vt: str = "d"):
    L = ref_lib(vt)
    m, n, nnz = C.c_long(), C.c_long(), C.c_long()
    rp, ci, va = C.c_void_p(), C.c_void_p(), C.c_void_p()
    L.ref_mtx_to_csr(os.fsencode(path), C.byref(m), C.byref(n), C.byref(nnz), C.byref(rp), C.byref(ci), C.byref(va))
    M, NNZ = m.value, nnz.value
    row_ptr = np.ctypeslib.as_array(C.cast(rp, C.POINTER(C.c_int32)), (M + 1,)).copy()
    col_idx = np.ctypeslib.as_array(C.cast(ci, C.POINTER(C.c_int32)), (max(NNZ, 1),))[:NNZ].copy()
    vals = np.ctypeslib.as_array(C.cast(va, C.POINTER(C.c_double)), (max(NNZ, 1),))[:NNZ].copy()
    for p in (rp, ci, va):
        L.ref_free(p)
    return M, n.value, row_ptr, col_idx, vals


def ref_partition(row_ptr, nnz: int, workers: int, pos: int, vt: str = "d") -> tuple[int, int]:
    s, e = C.c_long(), C.c_long()
    ref_lib(vt).ref_partition(row_ptr, len(row_ptr) - 1, nnz, workers, pos, C.byref(s), C.byref(e))
    return s.value, e.value


TWIN_FIELDS = ("nr_rows", "nr_cols", "avg_nnz_per_row", "std_nnz_per_row", "distribution", "placement", "bw",
               "skew", "avg_num_neighbours", "cross_row_similarity", "seed")


def ref_features(row_ptr, col_idx, ncols: int) -> dict:
    """The reference feature extractor (csr_matrix_features_validation, csr_util_gen.c:889-990) on a CSR pattern:
    the 11-field generator twin line it prints, parsed (plus the three 'extra features' of its first line)."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx if len(col_idx) else np.zeros(1), np.int32)
    buf = C.create_string_buffer(1 << 16)
    n = ref_lib("d").ref_features(rp, ci, len(rp) - 1, ncols, int(rp[-1]), buf, len(buf))
    if n < 0:
        raise RuntimeError("ref_features failed")
    text = buf.value.decode()
    twin = text[text.index("='") + 2:].split()
    out = {}
    for f, v in zip(TWIN_FIELDS, twin):
        out[f] = v if f in ("distribution", "placement") else (int(v) if f in ("nr_rows", "nr_cols", "seed") else float(v))
    extra = text[text.index("|") + 1:].split("|")[0].split()
    out["num_neigh_std"], out["cross_row_neigh_avg"], out["cross_row_neigh_std"] = (float(x) for x in extra)
    out["mem_footprint_mb"] = float(text.split("\n")[1].split()[0]) if "\n" in text else None
    return out


def ref_metrics(gold_d, test_d) -> np.ndarray:
    out = np.empty(8, np.float64)
    g = np.ascontiguousarray(gold_d, np.float64).ravel()
    t = np.ascontiguousarray(test_d, np.float64).ravel()
    ref_lib("d").ref_metrics(g, t, len(g), out)
    return out


# ---------------------------------------------------------------------------------------- sparse-attention pipeline
def sddmm(row_ptr, col_idx, mask_vals, Q, K, mode: int = 0) -> np.ndarray:
    """Pipeline SDDMM (sddmm_taco_naive.cpp:98-140): mode 0 = the reference's row-i-of-K product, 1 = Q K^T."""
    L = lib()
    dt = np.asarray(mask_vals).dtype
    m = len(row_ptr) - 1
    Q = np.ascontiguousarray(Q, dt)
    K = np.ascontiguousarray(K, dt)
    n = Q.shape[1]
    y = np.zeros(int(row_ptr[-1]), dt)
    fn = L.oracle_sddmm_d if dt == np.float64 else L.oracle_sddmm_f
    fn(np.ascontiguousarray(row_ptr, np.int32), np.ascontiguousarray(col_idx, np.int32),
       np.ascontiguousarray(mask_vals, dt), m, Q.ravel(), K.ravel(), n, mode, y)
    return y


def softmax(y: np.ndarray) -> np.ndarray:
    """The reference softmax over all nonzeros (sddmm_taco_naive.cpp:191-209), serial."""
    y = np.array(y, copy=True)
    (lib().oracle_softmax_d if y.dtype == np.float64 else lib().oracle_softmax_f)(y, len(y))
    return y


def spmm_rowmajor(row_ptr, col_idx, vals, ncols: int, x_rowmajor: np.ndarray) -> np.ndarray:
    """compute_csr's chain (spmm_kernel_csr.cpp:70-96) with B given row-major [ncols][n] (the pipeline's MKL
    layout): the same per-entry fma chain, the column-major view is just a transpose."""
    x = np.asarray(x_rowmajor)
    n = x.shape[1]
    return spmm(row_ptr, col_idx, vals, ncols, np.ascontiguousarray(x.T).ravel(), n)


def ref_smtx_read(path: str, vt: str = "d"):
    """The reference's DLMC reader (dlcm_matrix.c:258-324): (m, k, row_ptr, col_idx) as stored."""
    L = ref_lib(vt)
    m, k, nnz = C.c_long(), C.c_long(), C.c_long()
    rp, ci = C.c_void_p(), C.c_void_p()
    assert L.ref_smtx_read(path.encode(), C.byref(m), C.byref(k), C.byref(nnz), C.byref(rp), C.byref(ci)) == 0
    r = np.ctypeslib.as_array(C.cast(rp, C.POINTER(C.c_int32)), (m.value + 1,)).copy()
    c = np.ctypeslib.as_array(C.cast(ci, C.POINTER(C.c_int32)), (max(nnz.value, 1),))[:nnz.value].copy()
    L.ref_free(rp)
    L.ref_free(ci)
    return m.value, k.value, r, c
