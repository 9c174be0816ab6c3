"""GPU parity of the staged-rows kernel (spmm_staged_rows_kernel).

A staged workgroup gathers the B rows of its rows' next chunks with all 256 lanes into LDS, and one lane per
(row, column) folds them in CSR order: each C element is the reference's single left-to-right FMA chain
(compute_csr, spmm_kernel_csr.cpp:84-92), carried in a register across chunks.  So with staged rows forced
(SPMM_HIP_STAGED=1) every row the engine reports exact must be BIT-IDENTICAL to the oracle and to the row kernel
(SPMM_HIP_STAGED=-1); rows longer than T stay in the row kernel (pieces, normwise).  Covered: every B-row size the
kernel is built for (64 .. 1024 bytes: fp64 K = 8 .. 128, fp32 K = 16 .. 256), rows per workgroup 1 .. 32, K panels,
empty rows, a workgroup count that leaves empty slots, value updates, non-finite B, and the default policy.
"""
import numpy as np
import pytest

import spmm_amd as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, O


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64 if a.dtype == np.float64 else np.int32)


KEYS = ("SPMM_HIP_TILES", "SPMM_HIP_MFMA", "SPMM_HIP_STAGED", "SPMM_HIP_STAGED_R", "SPMM_HIP_STAGED_XCD",
        "SPMM_HIP_PANEL_K", "SPMM_HIP_SEQ_MAX")


def run(A, vals, x, k, monkeypatch, env, update=None):
    for kk in KEYS:
        monkeypatch.delenv(kk, raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    if update is not None:
        mf.update_values(update)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    ti, ex = mf.tile_info(), mf.exact_rows()
    mf.close()
    return y.reshape(A.m, k), ti, ex


def check(O, A, vals, x, k, y, ex):
    """Exact rows bit-identical to the oracle; the rest (pieces of rows > T) within the normwise contract."""
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
    assert np.array_equal(bits(y[ex]), bits(seq[ex]))
    if (~ex).any():
        g, absdot = O.gold(A.row_ptr, A.col_idx, vals.astype(np.float64), A.ncols, x.astype(np.float64), k)
        tol = 1e-10 if vals.dtype == np.float64 else 1e-3     # fp32 pieces: n * eps32 of the |a||b| sum
        assert O.normwise_ok(y[~ex].astype(np.float64), g[~ex], absdot[~ex], tol).all()


MATS = ["698 698 500 166.6667 normal random 0.05 0 0.05 0.05 14",      # small matrix of long rows
        "5588 5588 500 166.6667 normal random 0.3 100 0.95 0.95 14",   # long rows, similar
        "20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.95 3",     # a 20 K-nonzero row (row kernel) + short rows
        "3000 3000 100 33 normal random 0.6 0 0.5 0.05 14"]


@pytest.mark.parametrize("line", MATS, ids=["small", "similar", "split", "mid"])
@pytest.mark.parametrize("k,dt", [(8, "f64"), (16, "f64"), (32, "f64"), (64, "f64"), (128, "f64"),
                                  (16, "f32"), (32, "f32"), (64, "f32"), (256, "f32")])
def test_staged_bitexact(env, monkeypatch, line, k, dt):
    torch, O = env
    A = S.generate(S.gen_params(line))
    vals = A.values if dt == "f64" else A.values.astype(np.float32)
    x = O.drand48(11 + k, A.ncols * k) * 2.0 - 1.0
    if dt == "f32":
        x = x.astype(np.float32)
    y1, t1, ex1 = run(A, vals, x, k, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1"})
    assert t1["mode"] == "staged"
    y0, t0, ex0 = run(A, vals, x, k, monkeypatch, {"SPMM_HIP_STAGED": "-1", "SPMM_HIP_TILES": "-1"})
    assert t0["mode"] == "none"
    both = ex0 & ex1
    assert np.array_equal(bits(y1[both]), bits(y0[both]))
    assert ex1.sum() >= ex0.sum()            # staged rows are exact; vector lanes (inexact) only on the rest
    check(O, A, vals, x, k, y1, ex1)


@pytest.mark.parametrize("r", ["1", "2", "4", "8", "32"])
@pytest.mark.parametrize("k", [8, 32, 128])
def test_staged_rows_per_workgroup(env, monkeypatch, r, k):
    """Ragged rows (empty, 1, 3, chunk-boundary lengths, long) in workgroups of R rows, the last one partly empty."""
    torch, O = env
    rng = np.random.default_rng(5 + k)
    lens = np.array([0, 1, 3, 700, 0, 64, 65, 63, 8, 9, 511, 512, 513, 0, 2, 1000, 17, 33, 129, 255, 256, 257, 0,
                     4, 5, 6, 7, 128, 127, 1, 1, 300, 301, 2047, 31, 0, 40], np.int64)
    ncols = 3001
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    cols = np.concatenate([np.sort(rng.choice(ncols, size=int(n), replace=False)) for n in lens]).astype(np.int32)
    vals = rng.standard_normal(int(rp[-1]))
    A = S.CSR(rp, cols, vals, len(lens), ncols)
    x = rng.standard_normal(ncols * k)
    # T = 2048: every row whole (one staged chain each)
    y, t, ex = run(A, vals, x, k, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1",
                                                "SPMM_HIP_STAGED_R": r, "SPMM_HIP_SEQ_MAX": "2048"})
    assert t["mode"] == "staged" and ex.all()
    check(O, A, vals, x, k, y, ex)
    assert np.all(y[lens == 0] == 0.0)


@pytest.mark.parametrize("k", [64, 128])
def test_staged_k_panels(env, monkeypatch, k):
    """K panels of 32 columns (256-byte B rows) run one staged launch per panel."""
    torch, O = env
    A = S.generate(S.gen_params("5588 5588 500 166.6667 normal random 0.3 100 0.95 0.95 14"))
    x = O.drand48(3, A.ncols * k) * 2.0 - 1.0
    y, t, ex = run(A, A.values, x, k, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1",
                                                    "SPMM_HIP_PANEL_K": "32"})
    assert t["mode"] == "staged"
    check(O, A, A.values, x, k, y, ex)


def test_staged_xcd_order_same_bits(env, monkeypatch):
    torch, O = env
    A = S.generate(S.gen_params("5588 5588 500 166.6667 normal random 0.3 100 0.95 0.95 14"))
    x = O.drand48(4, A.ncols * 32)
    y1, _, _ = run(A, A.values, x, 32, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1"})
    y2, _, _ = run(A, A.values, x, 32, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1",
                                                     "SPMM_HIP_STAGED_XCD": "0"})
    assert np.array_equal(bits(y1), bits(y2))


def test_staged_value_update(env, monkeypatch):
    torch, O = env
    A = S.generate(S.gen_params("698 698 500 166.6667 normal random 0.05 0 0.05 0.05 14"))
    v2 = -A.values * 0.75 + 0.125
    x = O.drand48(9, A.ncols * 32) - 0.5
    y, t, ex = run(A, A.values, x, 32, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1"}, update=v2)
    assert t["mode"] == "staged"
    check(O, A, v2, x, 32, y, ex)


def test_staged_nonfinite_b(env, monkeypatch):
    """Inf / NaN in B reach exactly the rows that use those B rows, as in the reference's chain."""
    torch, O = env
    A = S.generate(S.gen_params("698 698 500 166.6667 normal random 0.05 0 0.05 0.05 14"))
    k = 32
    x = O.drand48(21, A.ncols * k) - 0.5
    x[5 * 1 + 3 * A.ncols] = np.inf          # column-major x: B[5][3] = inf, B[17][0] = nan
    x[17] = np.nan
    y, t, ex = run(A, A.values, x, k, monkeypatch, {"SPMM_HIP_STAGED": "1", "SPMM_HIP_TILES": "-1"})
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(bits(y[ex]), bits(seq[ex]))


def test_staged_policy_default(env, monkeypatch):
    """The default policy takes staged rows on a small long-row matrix (no environment), bit-exact."""
    torch, O = env
    A = S.generate(S.gen_params("698 698 500 166.6667 normal random 0.05 0 0.05 0.05 14"))
    x = O.drand48(2, A.ncols * 32) * 2.0 - 1.0
    y, t, ex = run(A, A.values, x, 32, monkeypatch, {})
    assert t["mode"] in ("staged", "mfma")
    check(O, A, A.values, x, 32, y, ex)
