"""GPU parity of the LDS x window (round 6; spmm_kernels.hpp spmm_rows_kernel XW).

At small K a block whose nonzeros' columns span few B rows stages that span of B (16-byte aligned, <= 16 KiB) in LDS
with the block, and its row groups gather from LDS instead of L2.  The values gathered and the FMA chain are the
same, so forced windows (SPMM_HIP_XWIN=1) must give output BIT-IDENTICAL to no windows (SPMM_HIP_XWIN=-1) on every row,
and the rows reported exact bit-identical to the oracle (reference compute_csr, spmm_kernel_csr.cpp:70-96; K = 1 is
the SpMV of spmv_kernel_csr.cpp:626-680): windowed and unwindowed blocks in one launch (a skewed row spans every
column), empty rows, split rows, vector lanes, paired rows, K of 1..16 including odd K (4- and 8-byte lanes), fp64 and
fp32, host-buffer and HBM-resident runs.
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


def run(S, A, vals, x, k, xw, monkeypatch, extra=None):
    monkeypatch.setenv("SPMM_HIP_XWIN", str(xw))
    for kk, vv in (extra or {}).items():
        monkeypatch.setenv(kk, vv)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    out = {"exact": mf.exact_rows(), "split": int(mf.info()[6])}
    mf.close()
    return y.reshape(A.m, k), out


def with_empty_rows(S, A, every):
    keep = np.ones(A.nnz, bool)
    for r in range(0, A.m, every):
        keep[A.row_ptr[r]:A.row_ptr[r + 1]] = False
    lens = np.diff(A.row_ptr).copy()
    lens[::every] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    return S.CSR(rp, A.col_idx[keep].copy(), A.values[keep].copy(), A.m, A.ncols)


MATS = {"band50": "20000 20000 50 16.6667 normal random 0.005 0 0.5 0.05 14",
        "band500": "6000 6000 500 166.6667 normal random 0.05 0 0.95 0.95 14",
        "narrow_skew": "8000 8000 20 6.6667 normal random 0.01 1000 0.5 0.5 14",   # a giant row spans every column
        "short": "50000 50000 5 1.6667 normal random 0.002 0 0.5 0.95 14"}


@pytest.mark.parametrize("name", list(MATS))
@pytest.mark.parametrize("k,dtype", [(1, "f64"), (2, "f64"), (3, "f64"), (4, "f64"), (8, "f64"),
                                     (1, "f32"), (4, "f32"), (8, "f32"), (16, "f32")])
def test_xwin_identical_and_oracle(env, monkeypatch, name, k, dtype):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[name]))
    if name == "short":
        A = with_empty_rows(S, A, 9)
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")      # every row one chain: rows are checked against the oracle exactly
    x = O.drand48(23 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y0, i0 = run(S, A, vals, xx, k, -1, monkeypatch)
    y1, i1 = run(S, A, vals, xx, k, 1, monkeypatch)
    monkeypatch.setenv("SPMM_HIP_XWIN", "1")
    p = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64 if dtype == "f64" else S.F32)
    # a 500-nonzero row spans >= 500 B rows: only at K = 1 (8- / 4-byte B rows) do its blocks fit 16 KiB
    assert p["xwin"] == (1 if name != "band500" or k == 1 else 0), p
    assert np.array_equal(i0["exact"], i1["exact"])
    assert np.array_equal(bits(y1), bits(y0))
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    ex = i1["exact"]
    assert ex.mean() > 0.5
    assert np.array_equal(bits(y1[ex]), bits(seq[ex]))
    if name == "short":
        empty = np.diff(A.row_ptr) == 0
        assert empty.sum() > 0 and (bits(y1[empty]) == 0).all()
    if name == "narrow_skew":
        assert i1["split"] >= 1
    if dtype == "f64" and (~ex).any():
        g, absdot = O.gold(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
        assert O.normwise_ok(y1[~ex], g[~ex], absdot[~ex], 1e-10).all()


@pytest.mark.parametrize("extra", [{}, {"SPMM_HIP_PAIR": "1"}, {"SPMM_HIP_FUSE": "0"}])
def test_xwin_with_other_modes(env, monkeypatch, extra):
    """Windows under the default lane policy (vector lanes at K = 1), forced pairing and the separate combine."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS["narrow_skew"]))
    for k in (1, 8):
        x = O.drand48(31 + k, A.ncols * k)
        y0, _ = run(S, A, A.values, x, k, -1, monkeypatch, extra)
        y1, i1 = run(S, A, A.values, x, k, 1, monkeypatch, extra)
        assert np.array_equal(bits(y1), bits(y0))
        seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
        ex = i1["exact"]
        assert np.array_equal(bits(y1[ex]), bits(seq[ex]))


@pytest.mark.parametrize("k", [1, 8])
def test_xwin_device_run(env, monkeypatch, k):
    """HBM-resident runs (spmm_hip_run_device), repeated launches on one handle."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS["band50"]))
    x = O.drand48(41, A.ncols * k)
    y_ref, _ = run(S, A, A.values, x, k, -1, monkeypatch)
    monkeypatch.setenv("SPMM_HIP_XWIN", "1")
    dev = torch.device("cuda", 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    B = torch.from_numpy(np.ascontiguousarray(x.reshape(k, A.ncols).T)).to(dev)
    Cd = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
    for _ in range(3):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    mf.close()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y_ref))
