"""GPU parity of the matrix-core tile kernel (spmm_mfma_tile_kernel).

The f64 MFMA (v_mfma_f64_16x16x4_f64) accumulates its four products in k order, each one fused multiply-add, and a
zero of the panel adds fma(+0, b, acc) == acc: every row of a matrix-core tile is the reference's left-to-right chain
(compute_csr, spmm_kernel_csr.cpp:70-96).  So with matrix-core tiles forced (SPMM_HIP_MFMA=1) every row the engine
reports exact must be BIT-IDENTICAL to the oracle and to the row kernel (SPMM_HIP_TILES=-1).  Also: K panels
(K = 64, 96, 128), non-finite B values (the chunk is recomputed by the sparse chain: the reference's Inf/NaN and
nothing more), value updates, duplicate columns / fp32 / narrow panels (refused: another kernel runs), the default
policy on a dense band, and a captured hipGraph replay.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, S, O


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64 if a.dtype == np.float64 else np.int32)


def handle(S, A, vals, k, monkeypatch, env):
    for kk in ("SPMM_HIP_TILES", "SPMM_HIP_MFMA", "SPMM_HIP_MFMA_REUSE"):
        monkeypatch.delenv(kk, raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    return S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)


def run(S, A, vals, x, k, monkeypatch, env):
    mf = handle(S, A, vals, k, monkeypatch, env)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    ti, ex = mf.tile_info(), mf.exact_rows()
    mf.close()
    return y.reshape(A.m, k), ti, ex


MATS = ["6000 6000 100 33 normal random 0.05 0 0.95 0.95 14",          # similar rows
        "3000 3000 300 100 normal random 0.05 10 1.4 0.5 14",          # dense narrow band
        "20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.95 3",     # a 20 K-nonzero split row + sparse tiles
        "4000 4000 40 13 normal random 0.6 0 0.05 0.05 14"]            # low reuse (density ~ 1/16)


@pytest.mark.parametrize("line", MATS, ids=["similar", "dense", "split", "lowreuse"])
@pytest.mark.parametrize("k", [32, 64, 96, 128])
def test_mfma_bitexact(env, monkeypatch, line, k):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(7 + k, A.ncols * k) * 2.0 - 1.0          # mixed signs: rounding in every chain
    y1, t1, ex1 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t1["mode"] == "mfma" and t1["tiles"] > 0
    y0, t0, ex0 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_TILES": "-1"})
    assert t0["tiles"] == 0
    both = ex0 & ex1
    assert both.sum() >= t1["rows"] * 0.99
    assert np.array_equal(bits(y1[both]), bits(y0[both]))
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(bits(y1[ex1]), bits(seq[ex1]))
    if (~ex1).any():
        g, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
        assert O.normwise_ok(y1[~ex1], g[~ex1], absdot[~ex1], 1e-10).all()


def test_mfma_nonfinite_b(env, monkeypatch):
    """Inf / NaN in B: a panel zero times them must not leak into rows that do not use those B rows."""
    torch, S, O = env
    A = S.generate(S.gen_params("6000 6000 100 33 normal random 0.05 0 0.95 0.95 14"))
    k = 32
    x = O.drand48(3, A.ncols * k).reshape(k, A.ncols)      # column-major: x[n][col]
    cols = np.unique(A.col_idx)
    rng = np.random.default_rng(4)
    x[rng.integers(0, k, 6), rng.choice(cols, 6)] = np.inf
    x[rng.integers(0, k, 6), rng.choice(cols, 6)] = -np.inf
    x[rng.integers(0, k, 6), rng.choice(cols, 6)] = np.nan
    x = x.reshape(-1)
    y1, t1, ex1 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t1["mode"] == "mfma"
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(np.isnan(y1[ex1]), np.isnan(seq[ex1]))
    fin = ~np.isnan(seq[ex1])
    assert np.array_equal(bits(y1[ex1][fin]), bits(seq[ex1][fin]))
    assert np.isfinite(seq).sum() > 0.9 * seq.size           # most rows never touch the planted values


def test_mfma_refused(env, monkeypatch):
    """fp32, 8-column panels and repeated columns never take matrix-core tiles (another kernel runs, still exact)."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[1]))
    for vals, k in ((A.values.astype(np.float32), 32), (A.values, 8)):
        mf = handle(S, A, vals, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
        assert mf.tile_info()["mode"] != "mfma"
        mf.close()
    # a repeated column in one row (duplicate .mtx entries are kept, not summed)
    rp, ci = A.row_ptr.copy(), A.col_idx.copy()
    ci[rp[5] + 1] = ci[rp[5]]
    B2 = S.CSR(rp, ci, A.values.copy(), A.m, A.ncols)
    x = O.drand48(5, A.ncols * 32)
    y, t, ex = run(S, B2, B2.values, x, 32, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t["mode"] != "mfma"
    seq = O.spmm(B2.row_ptr, B2.col_idx, B2.values, B2.ncols, x, 32)
    assert np.array_equal(bits(y[ex]), bits(seq[ex]))


def test_mfma_update_values(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[0]))
    k = 64
    x = O.drand48(6, A.ncols * k)
    mf = handle(S, A, A.values, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert mf.tile_info()["mode"] == "mfma"
    v2 = np.random.default_rng(9).uniform(-1, 1, A.nnz)
    mf.update_values(v2)
    y = np.zeros(A.m * k)
    mf.spmm(x, y, k)
    ex = mf.exact_rows()
    mf.close()
    want = O.spmm(A.row_ptr, A.col_idx, v2, A.ncols, x, k)
    assert np.array_equal(bits(y.reshape(A.m, k)[ex]), bits(want[ex]))


def test_mfma_policy_dense_band(env, monkeypatch):
    """Default policy: the 22354 x 500 dense band (16-row reuse ~ 5) takes matrix-core tiles at K = 32 and 128; a
    low-reuse matrix does not."""
    torch, S, O = env
    A = S.generate(S.gen_params("22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14"))
    for k in (32, 128):
        mf = handle(S, A, A.values, k, monkeypatch, {})
        assert mf.tile_info()["mode"] == "mfma", k
        mf.close()
    L = S.generate(S.gen_params("200000 200000 10 3.3333 normal random 0.6 0 0.05 0.05 14"))
    mf = handle(S, L, L.values, 32, monkeypatch, {})
    assert mf.tile_info()["mode"] != "mfma"
    mf.close()


def test_mfma_graph_replay(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[1]))
    k = 32
    mf = handle(S, A, A.values, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert mf.tile_info()["mode"] == "mfma"
    dev = torch.device("cuda", 0)
    B = torch.rand((A.ncols, k), dtype=torch.float64, device=dev)
    C1 = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    C2 = torch.empty_like(C1)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C1.data_ptr(), k, s.cuda_stream)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C2.data_ptr(), k, s.cuda_stream)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(C1.view(torch.int64), C2.view(torch.int64))
    mf.close()
