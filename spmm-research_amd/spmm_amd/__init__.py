"""spmm_amd -- Python host mirror of the reference's SpMM plugin surface, over the engine's C ABI.

The reference drives one kernel plugin per executable through ``csr_to_format(...)`` and ``MF->spmm(x, y, k)``
(benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h:9-30, spmm_kernel_csr.cpp:21-66).  This module exposes
the same surface on top of ``lib/libspmm_hip.so`` (include/spmm_hip.h) plus the host input path
``lib/libspmm_host.so`` (include/spmm_host.h: .mtx reader, coo_to_csr, synthetic generator, features,
CheckAccuracy).

There is no CPU fallback: if the HIP library is missing this module raises at import, and every compute call goes
to the GPU through the C ABI.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parents[1]          # spmm-research_amd/
LIB_DIR = PKG_ROOT / "lib"

F64, F32 = 0, 1
B_COL_MAJOR, B_ROW_MAJOR = 0, 1
SEQ_MAX = 2048      # upper bound of the per-handle split length (MatrixFormat.seq_max)
INFO_SLOTS = 20     # SPMM_HIP_INFO_SLOTS
STATUS = {0: "ok", -1: "invalid argument", -2: "out of memory", -3: "HIP runtime error", -4: "no such HIP device",
          -5: "k mismatch", -6: "malformed CSR", -7: "size overflow"}

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i64 = C.c_int64


class SpmmHipError(RuntimeError):
    def __init__(self, where: str, status: int, detail: str = ""):
        super().__init__(f"{where}: {STATUS.get(status, status)} ({status}) {detail}".rstrip())
        self.status = status


def _preload_hip_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm bundles its own libamdhip64 (DT_NEEDED "libamdhip64.so", found
    through its RPATH) while libspmm_hip.so needs "libamdhip64.so.7"; if the engine were loaded first the process
    would end up with two runtimes.  Preloading torch's copy (soname libamdhip64.so.7) makes both resolve to it.
    Set SPMM_HIP_RUNTIME=system to keep the system ROCm runtime instead."""
    if os.environ.get("SPMM_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec and spec.origin:
        rt = Path(spec.origin).parent / "lib" / "libamdhip64.so"
        if rt.exists():
            C.CDLL(str(rt), mode=C.RTLD_GLOBAL)


def _open(name: str) -> C.CDLL:
    path = LIB_DIR / name
    if not path.exists():
        raise ImportError(f"{path} is not built: run `make -C {PKG_ROOT}` (or __graft_entry__.build()); "
                          "the engine has no CPU fallback")
    return C.CDLL(str(path))


class _CSRStruct(C.Structure):
    _fields_ = [("m", _i64), ("ncols", _i64), ("nnz", _i64), ("row_ptr", C.POINTER(C.c_int32)),
                ("col_idx", C.POINTER(C.c_int32)), ("values", C.POINTER(C.c_double))]


class _GenParams(C.Structure):
    _fields_ = [("nr_rows", _i64), ("nr_cols", _i64), ("avg_nnz_per_row", C.c_double),
                ("std_nnz_per_row", C.c_double), ("distribution", C.c_char * 16), ("placement", C.c_char * 16),
                ("bw", C.c_double), ("skew", C.c_double), ("avg_num_neighbours", C.c_double),
                ("cross_row_similarity", C.c_double), ("seed", _i64)]


class _Features(C.Structure):
    _fields_ = [("distribution", C.c_char * 16), ("placement", C.c_char * 16), ("seed", _i64),
                ("nr_rows", _i64), ("nr_cols", _i64), ("nr_nzeros", _i64), ("density", C.c_double),
                ("mem_footprint", C.c_double), ("mem_range", C.c_char * 32),
                ("avg_nnz_per_row", C.c_double), ("std_nnz_per_row", C.c_double),
                ("avg_bw", C.c_double), ("std_bw", C.c_double), ("avg_bw_scaled", C.c_double),
                ("std_bw_scaled", C.c_double), ("avg_sc", C.c_double), ("std_sc", C.c_double),
                ("avg_sc_scaled", C.c_double), ("std_sc_scaled", C.c_double), ("skew", C.c_double),
                ("avg_num_neighbours", C.c_double), ("cross_row_similarity", C.c_double),
                ("max_nnz_per_row", _i64)]


class _Inspection(C.Structure):
    _fields_ = [("nv", _i64), ("nblk", _i64), ("nwin", _i64), ("nz", _i64), ("nlong", _i64), ("nslots", _i64),
                ("vrow_ptr", C.POINTER(C.c_int32)), ("vdest", C.POINTER(C.c_int32)), ("blk", C.POINTER(C.c_int32)),
                ("win_blk", C.POINTER(C.c_int32)), ("long_rows", C.POINTER(C.c_int32)),
                ("perm", C.POINTER(C.c_int64))]


class _Tiles(C.Structure):
    _fields_ = [("ntile", _i64), ("nchunk", _i64), ("ncol", _i64), ("nseg", _i64), ("nz", _i64), ("m", _i64),
                ("tiles", C.POINTER(C.c_int32)), ("chunks", C.POINTER(C.c_int32)), ("tcol", C.POINTER(C.c_int32)),
                ("tseg", C.POINTER(C.c_uint16)), ("tlidx", C.POINTER(C.c_uint16)), ("perm", C.POINTER(C.c_int64)),
                ("in_tile", C.POINTER(C.c_uint8))]


def _bind_hip(L: C.CDLL) -> C.CDLL:
    vp, i32, i64 = C.c_void_p, C.c_int32, _i64
    L.spmm_hip_create.argtypes = [_i32p, _i32p, vp, i64, i64, i64, i32, i32, i32, C.POINTER(vp)]
    L.spmm_hip_create_multi.argtypes = [_i32p, _i32p, vp, i64, i64, i64, i32, i32, i32, vp, C.POINTER(vp)]
    L.spmm_hip_ngpus.argtypes = [vp, C.POINTER(i32), C.POINTER(i32)]
    L.spmm_hip_shard.argtypes = [vp, i32, C.POINTER(i32), C.POINTER(i64), C.POINTER(i64), C.POINTER(vp)]
    L.spmm_hip_broadcast_b.argtypes = [vp, vp, i32, i32, vp]
    L.spmm_hip_run_sharded.argtypes = [vp, i32, vp]
    L.spmm_hip_run.argtypes = [vp, vp, vp, i32]
    L.spmm_hip_run_device.argtypes = [vp, vp, i32, vp, i32, vp]
    L.spmm_hip_run_device_batch.argtypes = [i32, C.POINTER(vp), C.POINTER(vp), C.POINTER(i32), C.POINTER(vp),
                                            C.POINTER(i32), vp]
    L.spmm_hip_plan.argtypes = [vp, i32]
    L.spmm_hip_last_times.argtypes = [vp, _f64p]
    L.spmm_hip_set_timing.argtypes = [vp, i32]
    L.spmm_hip_stats_labels.argtypes = [C.c_char_p, C.c_long]
    L.spmm_hip_stats.argtypes = [vp, C.c_char_p, C.c_long]
    L.spmm_hip_info.argtypes = [vp, np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")]
    L.spmm_hip_device_ptrs.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
    L.spmm_hip_exact_rows.argtypes = [vp, np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")]
    L.spmm_hip_destroy.argtypes = [vp]
    L.spmm_hip_partition_rows.argtypes = [_i32p, i64, i64, i64, i64, C.POINTER(i64), C.POINTER(i64)]
    L.spmm_hip_bytes_alg.argtypes = [i64, i64, i64, i32, i32]
    L.spmm_hip_bytes_alg.restype = C.c_double
    L.spmm_hip_debug_inspect.argtypes = [_i32p, _i32p, i64, i64, i32, i32, i64, C.POINTER(_Inspection)]
    L.spmm_hip_debug_free.argtypes = [C.POINTER(_Inspection)]
    L.spmm_hip_debug_free.restype = None
    L.spmm_hip_tile_info.argtypes = [vp, np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")]
    L.spmm_hip_tile_mode.argtypes = [vp]
    L.spmm_hip_run_rowmajor.argtypes = [vp, vp, vp, i32]
    L.spmm_hip_update_values.argtypes = [vp, vp]
    L.spmm_hip_update_values_device.argtypes = [vp, vp, vp]
    L.spmm_sddmm_create.argtypes = [_i32p, _i32p, vp, i64, i64, i64, i32, i32, i32, i32, C.POINTER(vp)]
    L.spmm_sddmm_run.argtypes = [vp, vp, vp, i64, vp]
    L.spmm_sddmm_run_device.argtypes = [vp, vp, vp, vp, vp]
    L.spmm_sddmm_destroy.argtypes = [vp]
    L.spmm_sddmm_last_error_detail.restype = C.c_char_p
    L.spmm_hip_debug_tiles.argtypes = [_i32p, _i32p, i64, i64, i32, i32, i32, i32, C.c_double, i32, i32,
                                       C.POINTER(_Tiles)]
    L.spmm_hip_debug_tiles_free.argtypes = [C.POINTER(_Tiles)]
    L.spmm_hip_debug_tiles_free.restype = None
    L.spmm_hip_debug_plan.argtypes = [_i32p, _i32p, i64, i64, i32, i32, i32, i32, _f64p]
    L.spmm_hip_debug_gate.argtypes = [i64, i64, i32, i32, i32, _f64p, _f64p]
    L.spmm_hip_strerror.argtypes = [C.c_int]
    L.spmm_hip_strerror.restype = C.c_char_p
    L.spmm_hip_last_error_detail.restype = C.c_char_p
    L.spmm_hip_device_count.argtypes = [C.POINTER(C.c_int)]
    L.spmm_hip_version.restype = C.c_char_p
    return L


def _bind_host(L: C.CDLL) -> C.CDLL:
    vp, i64 = C.c_void_p, _i64
    L.spmm_host_parse_gen_line.argtypes = [C.c_char_p, C.POINTER(_GenParams)]
    L.spmm_host_generate.argtypes = [C.POINTER(_GenParams), C.POINTER(_CSRStruct)]
    L.spmm_host_generate_row_ptr.argtypes = [C.POINTER(_GenParams), _i32p]
    L.spmm_host_generate_rows.argtypes = [C.POINTER(_GenParams), i64, i64, C.POINTER(_CSRStruct)]
    L.spmm_host_generate_masked.argtypes = [C.POINTER(_GenParams), np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS"),
                                            C.POINTER(_CSRStruct)]
    L.spmm_host_features.argtypes = [C.POINTER(_CSRStruct), C.POINTER(_Features)]
    L.spmm_host_mtx_read.argtypes = [C.c_char_p, C.POINTER(_CSRStruct), C.c_char_p, C.c_int, C.POINTER(C.c_int32)]
    L.spmm_host_smtx_read.argtypes = [C.c_char_p, i64, C.POINTER(_CSRStruct)]
    L.spmm_host_coo_to_csr.argtypes = [_i32p, _i32p, vp, i64, i64, i64, _i32p, _i32p, _f64p]
    L.spmm_host_csr_free.argtypes = [C.POINTER(_CSRStruct)]
    L.spmm_host_drand48_fill.argtypes = [i64, _f64p, i64]
    L.spmm_host_uniform_fill.argtypes = [i64, C.c_double, C.c_double, _f64p, i64]
    L.spmm_host_check_accuracy.argtypes = [_i32p, _i32p, _f64p, i64, i64, _f64p, C.c_int32, vp, C.c_int32,
                                           C.c_double, _f64p]
    return L


_preload_hip_runtime()
hip = _bind_hip(_open("libspmm_hip.so"))
host = _bind_host(_open("libspmm_host.so"))

def _detail() -> str:
    d = hip.spmm_hip_last_error_detail()
    return d.decode() if d else ""


def _check(where: str, st: int):
    if st != 0:
        raise SpmmHipError(where, st, _detail())


# ------------------------------------------------------------------------------------------------ host side
@dataclass
class CSR:
    row_ptr: np.ndarray   # int32 [m+1]
    col_idx: np.ndarray   # int32 [nnz]
    values: np.ndarray    # float64 [nnz] (csr_a_ref)
    m: int
    ncols: int

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1]) if len(self.row_ptr) else 0


def _take_csr(s: _CSRStruct) -> CSR:
    m, n, nnz = s.m, s.ncols, s.nnz
    rp = np.ctypeslib.as_array(s.row_ptr, (m + 1,)).copy()
    ci = np.ctypeslib.as_array(s.col_idx, (max(nnz, 1),))[:nnz].copy()
    va = np.ctypeslib.as_array(s.values, (max(nnz, 1),))[:nnz].copy()
    host.spmm_host_csr_free(C.byref(s))
    return CSR(rp, ci, va, m, n)


def gen_params(line: str | None = None, **kw) -> _GenParams:
    """Generator parameters from an 11-field line (the reference's argv order) and/or keywords."""
    p = _GenParams()
    if line is not None:
        st = host.spmm_host_parse_gen_line(line.encode(), C.byref(p))
        if st != 0:
            raise ValueError(f"cannot parse generator line {line!r}")
    for k, v in kw.items():
        setattr(p, k, v.encode() if isinstance(v, str) else v)
    return p


def generate(params: _GenParams) -> CSR:
    s = _CSRStruct()
    st = host.spmm_host_generate(C.byref(params), C.byref(s))
    if st != 0:
        raise RuntimeError(f"generator failed ({st})")
    return _take_csr(s)


def generate_row_ptr(params: _GenParams) -> np.ndarray:
    rp = np.empty(params.nr_rows + 1, np.int32)
    st = host.spmm_host_generate_row_ptr(C.byref(params), rp)
    if st != 0:
        raise RuntimeError(f"generator failed ({st})")
    return rp


def generate_rows(params: _GenParams, r0: int, r1: int) -> CSR:
    s = _CSRStruct()
    st = host.spmm_host_generate_rows(C.byref(params), r0, r1, C.byref(s))
    if st != 0:
        raise RuntimeError(f"generator failed ({st})")
    return _take_csr(s)


def generate_masked(params: _GenParams, mask: np.ndarray) -> CSR:
    """The whole matrix's row_ptr with the columns / values of the rows where mask is set only (others zero)."""
    s = _CSRStruct()
    st = host.spmm_host_generate_masked(C.byref(params), np.ascontiguousarray(mask, np.uint8), C.byref(s))
    if st != 0:
        raise RuntimeError(f"generator failed ({st})")
    return _take_csr(s)


def features(a: CSR) -> dict:
    s = _CSRStruct(a.m, a.ncols, a.nnz, a.row_ptr.ctypes.data_as(C.POINTER(C.c_int32)),
                   a.col_idx.ctypes.data_as(C.POINTER(C.c_int32)), a.values.ctypes.data_as(C.POINTER(C.c_double)))
    f = _Features()
    st = host.spmm_host_features(C.byref(s), C.byref(f))
    if st != 0:
        raise RuntimeError(f"features failed ({st})")
    out = {}
    for name, _t in _Features._fields_:
        v = getattr(f, name)
        out[name] = v.decode() if isinstance(v, bytes) else v
    return out


def mtx_read(path: str | os.PathLike) -> tuple[CSR, str, int]:
    """.mtx -> CSR with the indexing of the reference's mtx_read + coo_to_csr; returns (csr, field, symmetry)."""
    s = _CSRStruct()
    field = C.create_string_buffer(32)
    sym = C.c_int32()
    st = host.spmm_host_mtx_read(os.fsencode(str(path)), C.byref(s), field, 32, C.byref(sym))
    if st != 0:
        raise ValueError(f"cannot read {path} (status {st})")
    return _take_csr(s), field.value.decode(), sym.value


def smtx_read(path: str | os.PathLike, value_seed: int = 42) -> CSR:
    """DLMC .smtx -> CSR as the reference harness uses it (offsets and columns as stored, no sort); values are a
    seeded U[-1, 1) stream (the format has none; the reference's are time-seeded)."""
    s = _CSRStruct()
    st = host.spmm_host_smtx_read(os.fsencode(str(path)), value_seed, C.byref(s))
    if st != 0:
        raise ValueError(f"cannot read {path} (status {st})")
    return _take_csr(s)


def coo_to_csr(R, Cc, V, m: int, n: int | None = None) -> CSR:
    """coo_to_csr (csr_gen.c:163-217) with the reference's one-thread duplicate order; n = column count
    (default max column + 1)."""
    R = np.ascontiguousarray(R, np.int32)
    Cc = np.ascontiguousarray(Cc, np.int32)
    nnz = len(R)
    ncols = (int(Cc.max()) + 1 if nnz else 0) if n is None else int(n)
    rp = np.empty(m + 1, np.int32)
    ci = np.empty(max(nnz, 1), np.int32)
    va = np.empty(max(nnz, 1), np.float64)
    vptr = None if V is None else np.ascontiguousarray(V, np.float64).ctypes.data_as(C.c_void_p)
    st = host.spmm_host_coo_to_csr(R, Cc, vptr, m, ncols, nnz, rp, ci, va)
    if st != 0:
        raise ValueError(f"coo_to_csr failed ({st})")
    return CSR(rp, ci[:nnz], va[:nnz], m, ncols)


def drand48(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, np.float64)
    host.spmm_host_drand48_fill(seed, out, n)
    return out


def uniform(seed: int, lo: float, hi: float, n: int) -> np.ndarray:
    out = np.empty(n, np.float64)
    host.spmm_host_uniform_fill(seed, lo, hi, out, n)
    return out


def check_accuracy(a: CSR, x_ref_colmajor: np.ndarray, k: int, y_test: np.ndarray, eps: float) -> np.ndarray:
    """Harness CheckAccuracy (spmv_bench.cpp:121-206) + normwise check; see include/spmm_host.h for out[]."""
    out = np.empty(11, np.float64)
    y = np.ascontiguousarray(y_test)
    dt = 1 if y.dtype == np.float32 else 0
    host.spmm_host_check_accuracy(a.row_ptr, a.col_idx, np.ascontiguousarray(a.values, np.float64), a.m, a.ncols,
                                  np.ascontiguousarray(x_ref_colmajor, np.float64), k, y.ctypes.data_as(C.c_void_p),
                                  dt, eps, out)
    return out


def partition_rows(row_ptr: np.ndarray, nnz: int, workers: int, pos: int) -> tuple[int, int]:
    """loop_partitioner_balance_prefix_sums (lib/parallel_util.h:141-165): rows [s, e) of worker pos."""
    s, e = _i64(), _i64()
    _check("partition_rows", hip.spmm_hip_partition_rows(np.ascontiguousarray(row_ptr, np.int32),
                                                           len(row_ptr) - 1, nnz, workers, pos,
                                                           C.byref(s), C.byref(e)))
    return s.value, e.value


def bytes_alg(m: int, ncols: int, nnz: int, k: int, dtype: int = F64) -> float:
    return hip.spmm_hip_bytes_alg(m, ncols, nnz, k, dtype)


def debug_inspect(row_ptr: np.ndarray, col_idx: np.ndarray, ncols: int, T: int, cap: int,
                  win_cols: int = 0) -> dict:
    """The inspector's work decomposition (host only; spmm_hip_debug_inspect): virtual rows, destination codes,
    workgroup blocks, per-window block ranges, the window-major nonzero permutation and the split rows."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx if len(col_idx) else np.zeros(1), np.int32)
    ins = _Inspection()
    _check("debug_inspect", hip.spmm_hip_debug_inspect(rp, ci, len(rp) - 1, ncols, T, cap, win_cols, C.byref(ins)))
    try:
        def arr(p, n):
            return np.ctypeslib.as_array(p, (max(n, 1),))[:n].copy()
        out = {"vrow_ptr": arr(ins.vrow_ptr, ins.nv + 1), "vdest": arr(ins.vdest, ins.nv if (win_cols or ins.nslots) else 0),
               "blk": arr(ins.blk, 2 * ins.nblk).reshape(-1, 2), "win_blk": arr(ins.win_blk, ins.nwin + 1),
               "long_rows": arr(ins.long_rows, 4 * ins.nlong).reshape(-1, 4), "nslots": int(ins.nslots),
               "perm": arr(ins.perm, ins.nz) if ins.nz else None}
    finally:
        hip.spmm_hip_debug_free(C.byref(ins))
    return out


def debug_tiles(row_ptr: np.ndarray, col_idx: np.ndarray, ncols: int, T: int, rmax: int = 64, uc: int = 128,
                capa: int = 2048, min_reuse: float = 4.0, colmax: int = 0, dmax: int = 0) -> dict:
    """The tile decomposition (host only; spmm_hip_debug_tiles): tiles, chunks, union columns, per-chunk segment
    offsets, the chunk-major nonzero permutation (-1 = padding), chunk-local columns and the rows in tiles."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx if len(col_idx) else np.zeros(1), np.int32)
    t = _Tiles()
    _check("debug_tiles", hip.spmm_hip_debug_tiles(rp, ci, len(rp) - 1, ncols, T, rmax, uc, capa, min_reuse,
                                                   colmax, dmax, C.byref(t)))
    try:
        def arr(p, n):
            return np.ctypeslib.as_array(p, (max(n, 1),))[:n].copy()
        out = {"tiles": arr(t.tiles, 4 * t.ntile).reshape(-1, 4), "chunks": arr(t.chunks, 4 * (t.nchunk + 1)).reshape(-1, 4),
               "tcol": arr(t.tcol, t.ncol), "tseg": arr(t.tseg, t.nseg), "tlidx": arr(t.tlidx, t.nz),
               "perm": arr(t.perm, t.nz), "in_tile": arr(t.in_tile, t.m).astype(bool)}
    finally:
        hip.spmm_hip_debug_tiles_free(C.byref(t))
    return out


PLAN_SLOTS = 32     # SPMM_HIP_PLAN_SLOTS
PLAN_FIELDS = ("mode", "gate", "r16", "take", "est_tile_nnz", "est_chunks", "max_chunks", "t_on_us", "t_off_us",
               "sampled", "seq_max", "piece", "kw", "npanels", "ntile", "tile_nnz", "tile_chunks", "blocks",
               "split_rows", "exact_rows", "lmax", "xcd", "nwin", "gate_only", "fp_lo", "fp_hi", "est_tiles", "pair",
               "pair_reuse", "cap")
GATE_SAMPLE = ("sampled", "r16", "take", "est_tiles", "est_tile_nnz", "est_chunks", "max_chunks")


def debug_gate(m: int, nnz: int, k: int, sample: dict, dtype: int = F64) -> dict:
    """The matrix-core gate's cost model (spmm_hip_debug_gate) on a recorded gate sample (debug_plan's fields)."""
    v = np.array([float(sample[f]) for f in GATE_SAMPLE], np.float64)
    out = np.zeros(3, np.float64)
    _check("debug_gate", hip.spmm_hip_debug_gate(int(m), int(nnz), int(k), int(sample["kw"]), int(dtype), v, out))
    return {"gate": int(out[0]), "t_on_us": float(out[1]), "t_off_us": float(out[2])}


def debug_plan(row_ptr: np.ndarray, col_idx: np.ndarray, ncols: int, k: int, dtype: int = F64, mfma: int = 0,
               gate_only: bool = False) -> dict:
    """What spmm_hip_plan decides for (CSR, k, dtype), on the host (spmm_hip_debug_plan): tile mode, the matrix-core
    gate's sample and cost model, the plan's shape and a fingerprint of its tables.  mfma: the SPMM_HIP_MFMA override;
    gate_only: stop after the gate (col_idx only needs the gate's sampled rows, see gate_sample_rows)."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx if len(col_idx) else np.zeros(1), np.int32)
    out = np.zeros(PLAN_SLOTS, np.float64)
    _check("debug_plan", hip.spmm_hip_debug_plan(rp, ci, len(rp) - 1, ncols, k, dtype, mfma, int(gate_only), out))
    d = {f: float(out[i]) for i, f in enumerate(PLAN_FIELDS)}
    d["mode"] = {0: "none", 1: "lds", 2: "mfma"}[int(out[0])]
    d["fingerprint"] = int(out[25]) << 32 | int(out[24])
    return d


def gate_sample_rows(m: int) -> np.ndarray:
    """bool[m]: the rows of the matrix-core gate's sampled 16-row tiles (include/spmm_hip.h, spmm_hip_debug_plan)."""
    mask = np.zeros(m, np.uint8)
    nt = (m + 15) // 16
    ns = min(256, nt)
    for i in range(ns):
        t = i * nt // ns
        mask[t * 16:min(m, t * 16 + 16)] = 1
    return mask


def device_count() -> int:
    n = C.c_int()
    hip.spmm_hip_device_count(C.byref(n))
    return n.value


def stats_labels() -> str:
    buf = C.create_string_buffer(4096)
    w = hip.spmm_hip_stats_labels(buf, 4096)
    return buf.value[:max(w, 0)].decode()


# ------------------------------------------------------------------------------------------- plugin mirror
class MatrixFormat:
    """Mirror of ``struct Matrix_Format`` (spmv_kernel.h:9-26) backed by an engine handle on one GPU."""

    format_name = "HIP_CSR_MI355X"

    def __init__(self, row_ptr, col_ind, values, m: int, n: int, nnz: int, k: int = 0, device: int = 0,
                 ngpus: int = 1, devices=None):
        self.m, self.n, self.nnz = int(m), int(n), int(nnz)
        vals = np.ascontiguousarray(values)
        if vals.dtype not in (np.float64, np.float32):
            raise TypeError("values must be float64 or float32 (ValueType)")
        self.dtype = np.dtype(vals.dtype)
        self._dt = F64 if self.dtype == np.float64 else F32
        rp = np.ascontiguousarray(row_ptr, np.int32)
        ci = np.ascontiguousarray(col_ind, np.int32)
        if len(ci) == 0:
            ci = np.zeros(1, np.int32)
            vals = np.zeros(1, self.dtype)
        self._h = C.c_void_p()
        if ngpus > 1 or devices is not None:
            # multi-GPU handle (spmm_hip_create_multi): nnz-balanced row shards, one per device
            ng = int(ngpus if devices is None else len(devices))
            devs = None if devices is None else (C.c_int32 * ng)(*[int(d) for d in devices])
            _check("csr_to_format", hip.spmm_hip_create_multi(rp, ci, vals.ctypes.data_as(C.c_void_p), self.m, self.n,
                                                              self.nnz, int(k), self._dt, ng, devs, C.byref(self._h)))
        else:
            _check("csr_to_format", hip.spmm_hip_create(rp, ci, vals.ctypes.data_as(C.c_void_p), self.m, self.n,
                                                        self.nnz, int(k), self._dt, int(device), C.byref(self._h)))
        self.csr_mem_footprint = self.nnz * (self.dtype.itemsize + 4) + (self.m + 1) * 4
        self.mem_footprint = float(self.info()[7])

    # Matrix_Format::spmm(x, y, k): host x column-major [k][n], host y row-major [m][k] (overwritten)
    def spmm(self, x: np.ndarray, y: np.ndarray, k: int) -> None:
        if x.dtype != self.dtype or y.dtype != self.dtype:
            raise TypeError("x and y must have the handle's ValueType")
        if x.size < self.n * k or y.size < self.m * k or not (x.flags.c_contiguous and y.flags.c_contiguous):
            raise ValueError("x must hold n*k and y m*k contiguous values")
        _check("spmm", hip.spmm_hip_run(self._h, x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), k))

    def spmm_rowmajor(self, x: np.ndarray, y: np.ndarray, k: int) -> None:
        """Host x ROW-major [n][k] (the pipeline plugin's MKL layout), host y row-major [m][k]."""
        if x.dtype != self.dtype or y.dtype != self.dtype:
            raise TypeError("x and y must have the handle's ValueType")
        if x.size < self.n * k or y.size < self.m * k or not (x.flags.c_contiguous and y.flags.c_contiguous):
            raise ValueError("x must hold n*k and y m*k contiguous values")
        _check("spmm_rowmajor", hip.spmm_hip_run_rowmajor(self._h, x.ctypes.data_as(C.c_void_p),
                                                          y.ctypes.data_as(C.c_void_p), k))

    def update_values(self, vals: np.ndarray) -> None:
        """Replace A's values (same pattern), host array."""
        v = np.ascontiguousarray(vals, self.dtype)
        if v.size < self.nnz:
            raise ValueError("need nnz values")
        _check("update_values", hip.spmm_hip_update_values(self._h, v.ctypes.data_as(C.c_void_p)))

    def update_values_device(self, d_vals: int, stream: int = 0) -> None:
        _check("update_values_device", hip.spmm_hip_update_values_device(self._h, C.c_void_p(d_vals),
                                                                         C.c_void_p(stream)))

    def spmm_device(self, d_b: int, b_layout: int, d_c: int, k: int, stream: int = 0) -> None:
        """HBM-resident run: d_b / d_c are device addresses (e.g. torch tensor .data_ptr())."""
        _check("spmm_device", hip.spmm_hip_run_device(self._h, C.c_void_p(d_b), b_layout, C.c_void_p(d_c), k,
                                                      C.c_void_p(stream)))

    def ngpus(self) -> tuple[int, int]:
        """(shards, broadcast mode: 0 peer copies, 1 RCCL)."""
        n, b = C.c_int32(), C.c_int32()
        _check("ngpus", hip.spmm_hip_ngpus(self._h, C.byref(n), C.byref(b)))
        return n.value, b.value

    def shard(self, g: int) -> dict:
        """Shard g of the handle: device, C rows [row0, row1), device-local C buffer address."""
        d, r0, r1, c = C.c_int32(), _i64(), _i64(), C.c_void_p()
        _check("shard", hip.spmm_hip_shard(self._h, g, C.byref(d), C.byref(r0), C.byref(r1), C.byref(c)))
        return {"device": d.value, "row0": r0.value, "row1": r1.value, "d_c": c.value or 0}

    def broadcast_b(self, d_b: int, b_layout: int, k: int, stream: int = 0) -> None:
        _check("broadcast_b", hip.spmm_hip_broadcast_b(self._h, C.c_void_p(d_b), b_layout, k, C.c_void_p(stream)))

    def run_sharded(self, k: int, stream: int = 0) -> None:
        _check("run_sharded", hip.spmm_hip_run_sharded(self._h, k, C.c_void_p(stream)))

    def plan(self, k: int) -> None:
        _check("plan", hip.spmm_hip_plan(self._h, k))

    def last_times(self) -> dict:
        t = np.zeros(4, np.float64)
        _check("last_times", hip.spmm_hip_last_times(self._h, t))
        return {"kernel_ms": t[0], "transpose_ms": t[1], "h2d_ms": t[2], "d2h_ms": t[3]}

    def info(self) -> np.ndarray:
        out = np.zeros(INFO_SLOTS, np.int64)
        _check("info", hip.spmm_hip_info(self._h, out))
        return out

    def tile_info(self) -> dict:
        """LDS B tiles of the current plan (spmm_hip_tile_info)."""
        out = np.zeros(7, np.int64)
        _check("tile_info", hip.spmm_hip_tile_info(self._h, out))
        mode = hip.spmm_hip_tile_mode(self._h)
        return {"tiles": int(out[0]), "rows": int(out[1]), "nnz": int(out[2]), "chunks": int(out[3]),
                "reuse": out[4] / 1000.0, "xcd": int(out[5]), "wide": int(out[6]),
                "mode": {0: "none", 1: "lds", 2: "mfma"}.get(mode, "none")}

    def exact_rows(self) -> np.ndarray:
        """bool[m]: rows computed as the reference's single left-to-right FMA chain (bit-identical to it)."""
        mask = np.zeros(max(self.m, 1), np.uint8)
        _check("exact_rows", hip.spmm_hip_exact_rows(self._h, mask))
        return mask[:self.m].astype(bool)

    @property
    def seq_max(self) -> int:
        """Split length T of the current plan: rows with <= T nonzeros are bit-identical to the reference."""
        return int(self.info()[8])

    def statistics_start(self) -> None:
        """Matrix_Format::statistics_start (spmv_kernel.h:19): later spmm_device calls record timing events."""
        _check("set_timing", hip.spmm_hip_set_timing(self._h, 1))

    def statistics_print_data(self) -> str:
        buf = C.create_string_buffer(4096)
        w = hip.spmm_hip_stats(self._h, buf, 4096)
        if w < 0:
            raise SpmmHipError("stats", w, _detail())
        return buf.value.decode()

    def close(self) -> None:
        if self._h:
            hip.spmm_hip_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_device_batch(entries, stream: int = 0) -> None:
    """Independent HBM-resident SpMMs of different handles, run concurrently (spmm_hip_run_device_batch): entries =
    [(MatrixFormat, d_b, b_layout, d_c, k), ...]; the first runs on `stream`, the rest on forked side streams joined
    back into it (graph-capturable)."""
    n = len(entries)
    hs = (C.c_void_p * n)(*[e[0]._h for e in entries])
    bs = (C.c_void_p * n)(*[e[1] for e in entries])
    lay = (C.c_int32 * n)(*[e[2] for e in entries])
    cs = (C.c_void_p * n)(*[e[3] for e in entries])
    ks = (C.c_int32 * n)(*[e[4] for e in entries])
    _check("run_device_batch", hip.spmm_hip_run_device_batch(n, hs, bs, lay, cs, ks, C.c_void_p(stream)))


def csr_to_format(row_ptr, col_ind, values, m: int, n: int, nnz: int, k: int = 0, device: int = 0, ngpus: int = 1,
                  devices=None) -> MatrixFormat:
    """Factory with the reference's signature (spmv_kernel.h:29); ngpus / devices: a multi-GPU handle."""
    return MatrixFormat(row_ptr, col_ind, values, m, n, nnz, k, device, ngpus, devices)


def statistics_print_labels() -> str:
    return stats_labels()
