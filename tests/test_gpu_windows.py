"""GPU parity of the column-window (chained) mode against the plain mode and the oracle.

In chained mode each column window is one launch and every row's FMA chain continues through C from window to
window (spmm_kernels.hpp DEST_CHAIN), so the output must be BIT-IDENTICAL to the plain single-launch mode for every
row -- split rows included, since their T-pieces are chained the same way before the same combine -- and rows of
<= T nonzeros bit-identical to the oracle (reference compute_csr, spmm_kernel_csr.cpp:70-96).
SPMM_HIP_WIN_BYTES=<bytes of B per window> forces windows, -1 disables them.
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


def run(S, A, vals, x, k, win_bytes, monkeypatch):
    monkeypatch.setenv("SPMM_HIP_WIN_BYTES", str(win_bytes))
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    inf = mf.info()
    ex = mf.exact_rows()
    mf.close()
    return y.reshape(A.m, k), {"T": int(inf[8]), "windows": int(inf[12]), "win_cols": int(inf[13]),
                               "segments": int(inf[14]), "panels": int(inf[11]), "lmax": int(inf[16]), "exact": ex}


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64 if a.dtype == np.float64 else np.int32)


MATS = ["20000 16000 40 13.3333 normal random 0.3 50 0.95 0.5 14",     # plain rows
        "20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.5 3",      # one 20 K-nonzero row: split + chained
        "3000 3000 300 100 normal random 0.05 10 1.4 0.95 14"]         # dense narrow band


@pytest.mark.parametrize("line", MATS, ids=["plain", "split", "dense"])
@pytest.mark.parametrize("k", [1, 8, 32, 33, 128])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_windows_identical_to_plain(env, monkeypatch, line, k, dtype):
    torch, S, O = env
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")       # vector lanes depend on block composition
    A = S.generate(S.gen_params(line))
    x = O.drand48(11 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y0, i0 = run(S, A, vals, xx, k, -1, monkeypatch)
    assert i0["windows"] == 1
    for wb in (4096, 300_000, 2 << 20):
        y1, i1 = run(S, A, vals, xx, k, wb, monkeypatch)
        wcols = max(1, wb // (k * vals.itemsize))        # no K panels at these sizes
        assert i1["windows"] == ((A.ncols + wcols - 1) // wcols if wcols < A.ncols else 1), (wb, i1)
        assert i1["T"] == i0["T"]
        assert np.array_equal(bits(y1), bits(y0)), (wb, i1)
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    short = i0["exact"]
    assert np.array_equal(bits(y0[short]), bits(seq[short]))


@pytest.mark.parametrize("line", MATS[:2], ids=["plain", "split"])
@pytest.mark.parametrize("k", [1, 32])
def test_xcd_order_identical(env, monkeypatch, line, k):
    """XCD-contiguous block order only moves workgroups between XCDs: same bits."""
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(3 + k, A.ncols * k)
    monkeypatch.setenv("SPMM_HIP_XCD", "-1")
    y0, _ = run(S, A, A.values, x, k, -1, monkeypatch)
    monkeypatch.setenv("SPMM_HIP_XCD", "1")
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    assert mf.info()[15] == 1
    y1 = np.full(A.m * k, np.nan)
    mf.spmm(x, y1, k)
    mf.close()
    assert np.array_equal(bits(y1.reshape(A.m, k)), bits(y0))


@pytest.mark.parametrize("line", MATS, ids=["plain", "split", "dense"])
@pytest.mark.parametrize("k", [1, 8, 32, 33])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_vector_lanes(env, monkeypatch, line, k, dtype):
    """Vector lanes (several lane groups per long row, fixed shuffle tree): rows the engine reports exact equal the
    oracle bit for bit, the others are within the normwise bound and identical run to run; with and without
    column windows."""
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(21 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    g, absdot = O.gold(A.row_ptr, A.col_idx, vals.astype(np.float64), A.ncols, xx.astype(np.float64), k)
    deg = np.diff(A.row_ptr)
    monkeypatch.setenv("SPMM_HIP_LANES", "64")
    for wb in (-1, 300_000):
        y1, i1 = run(S, A, vals, xx, k, wb, monkeypatch)
        y2, _ = run(S, A, vals, xx, k, wb, monkeypatch)
        assert np.array_equal(bits(y1), bits(y2)), "vector lanes must be deterministic"
        assert i1["lmax"] > 1 or k == 33       # K=33: 64-lane row groups already fill a wavefront (cap 64/G = 1)
        ex = i1["exact"]
        assert np.array_equal(bits(y1[ex]), bits(seq[ex]))
        if dtype == "f64":
            assert O.normwise_ok(y1, g, absdot, 1e-10).all()
        else:
            tol = (np.maximum(deg, 1)[:, None] + 1) * 2.0 ** -24 * 1.01
            assert (np.abs(y1.astype(np.float64) - g) <= tol * np.maximum(np.abs(g), absdot)).all()


def test_policy_windows_dense_matrix(env, monkeypatch):
    """The inspector picks windows on its own for dense rows whose column span is several L2s of B rows wide
    (K=32 fp64: span 60 K columns = 15 MB of B rows, 300 nonzeros per row)."""
    torch, S, O = env
    A = S.generate(S.gen_params("100000 100000 300 100 normal random 0.6 10 0.95 0.5 14"))
    k = 32
    x = O.drand48(3, A.ncols * k)
    monkeypatch.delenv("SPMM_HIP_WIN_BYTES", raising=False)
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")       # split-row pieces would get block-dependent lanes
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    y = np.full(A.m * k, np.nan)
    mf.spmm(x, y, k)
    inf = mf.info()
    mf.close()
    assert inf[12] > 1, inf
    y0, _ = run(S, A, A.values, x, k, -1, monkeypatch)
    assert np.array_equal(bits(y.reshape(A.m, k)), bits(y0))


def test_windows_device_path_and_graph_capture(env, monkeypatch):
    """Chained launches are stream-ordered: device path (row-major and col-major B) and a captured hipGraph replay
    give the host path's bits."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[2]))
    k = 32
    x = O.drand48(5, A.ncols * k)
    y_host, inf = run(S, A, A.values, x, k, 1 << 16, monkeypatch)
    assert inf["windows"] > 1
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    dev = torch.device("cuda", 0)
    Bc = torch.from_numpy(x).to(dev)
    Br = torch.from_numpy(x.reshape(k, A.ncols).T.copy()).to(dev)
    Cd = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        mf.spmm_device(Br.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, s.cuda_stream)
    s.synchronize()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y_host))
    Cd.fill_(float("nan"))
    mf.spmm_device(Bc.data_ptr(), S.B_COL_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y_host))
    g = torch.cuda.CUDAGraph()
    Cd.fill_(float("nan"))
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        mf.spmm_device(Br.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y_host))
    mf.close()
