"""GPU parity of the LDS B tile mode (spmm_tile_kernel).

Every tile row is one left-to-right FMA chain in CSR order, so with tiles forced (SPMM_HIP_TILES=1) every row the
engine reports exact must be BIT-IDENTICAL to the oracle (reference compute_csr, spmm_kernel_csr.cpp:70-96) and to
the row-kernel-only plan (SPMM_HIP_TILES=-1); the others (split rows left to the row kernel) within the normwise
1e-10 (fp64) / (n+1)*2^-24 (fp32) bound.  Covers K panels (last panel narrower), empty rows inside tiles, duplicate
columns, rows too long for a tile, unsorted rows (tiles refused) and a captured hipGraph replay.
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


@pytest.fixture(autouse=True)
def sparse_tile_kernel(monkeypatch):
    """These tests cover the sparse LDS tile kernel; fp64 32-column panels would otherwise take the matrix-core tile
    kernel (tests/test_gpu_mfma.py)."""
    monkeypatch.setenv("SPMM_HIP_MFMA", "-1")


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64 if a.dtype == np.float64 else np.int32)


def run(S, A, vals, x, k, tiles, monkeypatch, extra=None):
    monkeypatch.setenv("SPMM_HIP_TILES", str(tiles))
    for kk, vv in (extra or {}).items():
        monkeypatch.setenv(kk, vv)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    ti, ex, inf = mf.tile_info(), mf.exact_rows(), mf.info()
    mf.close()
    return y.reshape(A.m, k), ti, ex, inf


def check(O, A, vals, x, k, y, ex):
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
    assert np.array_equal(bits(y[ex]), bits(seq[ex]))
    if (~ex).any():
        g, absdot = O.gold(A.row_ptr, A.col_idx, vals.astype(np.float64), A.ncols, x.astype(np.float64), k)
        if vals.dtype == np.float64:
            assert O.normwise_ok(y[~ex], g[~ex], absdot[~ex], 1e-10).all()
        else:
            lens = np.diff(A.row_ptr)[~ex][:, None]
            err = np.abs(y[~ex].astype(np.float64) - g[~ex])
            assert np.all(err <= (lens + 1) * 2.0 ** -24 * absdot[~ex] + 1e-30)


MATS = ["6000 6000 100 33 normal random 0.05 0 0.95 0.95 14",          # similar rows: every tile taken
        "3000 3000 300 100 normal random 0.05 10 1.4 0.5 14",          # dense narrow band
        "20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.95 3"]    # a 20 K-nonzero split row + tiles


@pytest.mark.parametrize("line", MATS, ids=["similar", "dense", "split"])
@pytest.mark.parametrize("k", [8, 16, 32, 64, 128])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_tiles_bitexact(env, monkeypatch, line, k, dtype):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(5 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y1, t1, ex1, _ = run(S, A, vals, xx, k, 1, monkeypatch)
    if k * vals.itemsize < 64:                      # B rows under 64 bytes never take tiles
        assert t1["tiles"] == 0
    else:
        assert t1["tiles"] > 0 and t1["rows"] > 0
    y0, t0, ex0, _ = run(S, A, vals, xx, k, -1, monkeypatch)
    assert t0["tiles"] == 0
    both = ex0 & ex1
    assert np.array_equal(bits(y1[both]), bits(y0[both]))
    check(O, A, vals, xx, k, y1, ex1)


@pytest.mark.parametrize("k,panel", [(96, 32), (128, 64), (64, 16), (80, 32)])
def test_tiles_k_panels(env, monkeypatch, k, panel):
    """K panels (one tile launch per panel) with tiles forced; tiles need equal panels (K % panel == 0) and
    power-of-two B rows, otherwise the row kernel computes everything."""
    torch, S, O = env
    A = S.generate(S.gen_params("5000 5000 60 20 normal random 0.1 0 0.95 0.95 14"))
    x = O.drand48(9, A.ncols * k)
    y, t, ex, inf = run(S, A, A.values, x, k, 1, monkeypatch, {"SPMM_HIP_PANEL_K": str(panel)})
    assert inf[11] == (k + panel - 1) // panel
    assert (t["tiles"] > 0) == (k % panel == 0)
    check(O, A, A.values, x, k, y, ex)


def test_tiles_edge_rows(env, monkeypatch):
    """Empty rows inside tiles, duplicate columns, one row longer than T (row kernel), a near-full column."""
    torch, S, O = env
    rng = np.random.default_rng(4)
    m, n = 4000, 300
    lens = rng.integers(0, 40, m)
    lens[100:180] = 0
    lens[2500] = 5000
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.concatenate([np.sort(rng.integers(0, n, L)) for L in lens]).astype(np.int32)
    col[rp[3000]:rp[3064]] = 7                      # 64 rows all on one column (a chunk of one column)
    col[rp[3000]:rp[3064]].sort()
    vals = rng.uniform(-1, 1, len(col))
    vals[::17] = -0.0
    A = S.CSR(rp, col, vals, m, n)
    for k in (8, 32):
        x = O.drand48(k, n * k)
        y, t, ex, _ = run(S, A, vals, x, k, 1, monkeypatch)
        assert t["tiles"] > 0 and not ex[2500]
        check(O, A, vals, x, k, y, ex)
        assert np.all(y[100:180] == 0)


def test_tiles_refused_unsorted(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params("3000 3000 100 33 normal random 0.05 0 0.95 0.95 14"))
    col = A.col_idx.copy()
    r = 1500
    col[A.row_ptr[r]:A.row_ptr[r + 1]] = col[A.row_ptr[r]:A.row_ptr[r + 1]][::-1].copy()
    B = S.CSR(A.row_ptr, col, A.values, A.m, A.ncols)
    x = O.drand48(1, A.ncols * 32)
    y, t, ex, _ = run(S, B, B.values, x, 32, 1, monkeypatch)
    assert t["tiles"] == 0
    check(O, B, B.values, x, 32, y, ex)


def test_tiles_graph_replay(env, monkeypatch):
    """The two launches (row kernel for the residual rows, tile kernel) captured in a hipGraph replay identically."""
    torch, S, O = env
    monkeypatch.setenv("SPMM_HIP_TILES", "1")
    A = S.generate(S.gen_params("20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.95 3"))
    k = 32
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    assert mf.tile_info()["tiles"] > 0
    dev = torch.device("cuda", 0)
    x = O.drand48(2, A.ncols * k)
    B = torch.from_numpy(x.reshape(k, A.ncols).T.copy()).to(dev)
    C1 = torch.zeros((A.m, k), dtype=torch.float64, device=dev)
    C2 = torch.zeros_like(C1)
    s = torch.cuda.Stream(dev)
    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C1.data_ptr(), k, s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C2.data_ptr(), k, s.cuda_stream)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(C1.view(torch.int64), C2.view(torch.int64))
    mf.close()


def test_tile_policy_gates(env, monkeypatch):
    """The default policy: tiles need sampled reuse >= 8 AND >= 512 candidate tiles.  A small dense
    matrix (2,445 rows, 77 candidate tiles) stays with the row kernel even though its reuse is high; a large
    high-reuse band takes tiles; both stay exact where the engine says so."""
    torch, S, O = env
    monkeypatch.delenv("SPMM_HIP_TILES", raising=False)
    k = 32
    for line, want in (("2445 2445 500 166.6667 normal random 0.05 10000 0.95 0.95 14", False),
                       ("22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14", True)):
        A = S.generate(S.gen_params(line))
        x = np.random.default_rng(1).uniform(0, 1, A.ncols * k)          # the reference's column-major x
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
        y = np.full(A.m * k, np.nan)
        mf.spmm(x, y, k)
        ti, ex = mf.tile_info(), mf.exact_rows()
        mf.close()
        assert (ti["tiles"] > 0) == want, (line, ti)
        rows = np.random.default_rng(2).choice(A.m, 300, replace=False)
        sub = S.CSR(np.concatenate([[0], np.cumsum(np.diff(A.row_ptr)[rows])]).astype(np.int32),
                    np.concatenate([A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows]),
                    np.concatenate([A.values[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows]), len(rows), A.ncols)
        ys = y.reshape(A.m, k)[rows]
        seq = O.spmm(sub.row_ptr, sub.col_idx, sub.values, A.ncols, x, k)
        assert np.array_equal(bits(ys[ex[rows]]), bits(seq[ex[rows]]))


@pytest.mark.parametrize("line", MATS[:2], ids=["similar", "dense"])
@pytest.mark.parametrize("k", [16, 32, 64, 128])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("sw", [2, 4])
def test_tiles_wide_lanes_bitexact(env, monkeypatch, line, k, dtype, sw):
    """Wide compute lanes (SPMM_HIP_TILE_WIDE=S: S 16-byte pieces of a B row per lane, 1/S the lanes per row, same
    tile geometry) compute the same FMA chains: bit-identical to 16-byte lanes and to the oracle.  The width drops
    to what the rows per group allow (B rows >= 128 B for S=2); S=4 (measured slower) is no longer built: asking
    for it gives S=2."""
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(11 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y1, t1, ex1, _ = run(S, A, vals, xx, k, 1, monkeypatch, {"SPMM_HIP_TILE_WIDE": str(sw)})
    y0, t0, ex0, _ = run(S, A, vals, xx, k, 1, monkeypatch, {"SPMM_HIP_TILE_WIDE": "1"})
    assert t1["tiles"] > 0 and t0["tiles"] == t1["tiles"] and t0["wide"] == 1
    rb = k * vals.itemsize
    assert t1["wide"] == (2 if rb >= 128 else 1)
    assert np.array_equal(ex0, ex1)
    assert np.array_equal(bits(y1), bits(y0))
    check(O, A, vals, xx, k, y1, ex1)


def test_tile_policy_row_bytes(env, monkeypatch):
    """The default policy stages B rows of at most 256 bytes: the same high-reuse band that takes
    tiles at K=32 fp64 (256-B rows) keeps the row kernel at K=64 (512-B rows measured 6-26 % slower in tiles) and
    at K=64 fp32 (256-B rows) takes them again; forcing still tiles any eligible shape."""
    torch, S, O = env
    monkeypatch.delenv("SPMM_HIP_TILES", raising=False)
    A = S.generate(S.gen_params("22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14"))
    for k, vals, want in ((32, A.values, True), (64, A.values, False), (64, A.values.astype(np.float32), True)):
        mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
        assert (mf.tile_info()["tiles"] > 0) == want, (k, vals.dtype)
        mf.close()
    monkeypatch.setenv("SPMM_HIP_TILES", "1")
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, 64, 0)
    assert mf.tile_info()["tiles"] > 0
    mf.close()
