"""GPU parity of the wide block window (round 6; spmm_rows_kernel with CAP = 4096).

SPMM_HIP_CAP=4096 lets the inspector pack blocks of up to 4,096 nonzeros (twice the default LDS window) where the row
kernel has 16-byte lanes and row groups of >= 8 lanes, so a block of 500-nonzero rows holds ~8 rows for its row
groups instead of ~3.5.  Block boundaries move; every row is still ONE fused multiply-add chain from 0 in CSR order,
so the output must be BIT-IDENTICAL to the default window on every row, and the rows reported exact bit-identical to
the oracle (reference compute_csr, spmm_kernel_csr.cpp:70-96): long rows, split rows (fused and separate combine),
lanes past K, fp64 and fp32, host-buffer and HBM-resident runs.
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


def run(S, A, vals, x, k, cap, monkeypatch, extra=None):
    monkeypatch.setenv("SPMM_HIP_CAP", str(cap or 2048))   # 2048: the default window (the policy may pick 4096)
    for kk, vv in (extra or {}).items():
        monkeypatch.setenv(kk, vv)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    out = {"exact": mf.exact_rows(), "split": int(mf.info()[6]), "blocks": int(mf.info()[5])}
    mf.close()
    return y.reshape(A.m, k), out


MATS = {"avg500": "9000 9000 500 166.6667 normal random 0.3 0 0.5 0.05 14",
        "avg100_skew": "30000 30000 100 33.3333 normal random 0.3 1000 0.5 0.05 14",
        "avg50": "40000 40000 50 16.6667 normal random 0.6 0 0.05 0.05 14"}


@pytest.mark.parametrize("name", list(MATS))
@pytest.mark.parametrize("k,dtype", [(32, "f64"), (40, "f64"), (64, "f64"), (128, "f64"), (32, "f32"), (64, "f32")])
def test_widecap_identical_and_oracle(env, monkeypatch, name, k, dtype):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[name]))
    monkeypatch.setenv("SPMM_HIP_MFMA", "-1")
    monkeypatch.setenv("SPMM_HIP_TILES", "-1")
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")
    x = O.drand48(29 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y0, i0 = run(S, A, vals, xx, k, 0, monkeypatch)
    y1, i1 = run(S, A, vals, xx, k, 4096, monkeypatch)
    assert i1["blocks"] < i0["blocks"], (i0, i1)          # the wide window packed more rows per block
    assert np.array_equal(i0["exact"], i1["exact"])
    assert np.array_equal(bits(y1), bits(y0))
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    ex = i1["exact"]
    assert ex.mean() > 0.99
    assert np.array_equal(bits(y1[ex]), bits(seq[ex]))
    if name == "avg100_skew":
        assert i1["split"] >= 1


@pytest.mark.parametrize("extra", [{}, {"SPMM_HIP_FUSE": "0"}])
def test_widecap_default_lanes_and_combine(env, monkeypatch, extra):
    """The default lane policy and both combines with the wide window; repeated device launches."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS["avg100_skew"]))
    k = 32
    x = O.drand48(37, A.ncols * k)
    monkeypatch.setenv("SPMM_HIP_MFMA", "-1")
    y0, i0 = run(S, A, A.values, x, k, 0, monkeypatch, extra)
    y1, i1 = run(S, A, A.values, x, k, 4096, monkeypatch, extra)
    # a split row's pieces may take vector lanes by how many pieces share a block, which the window changes: only the
    # rows both runs report exact must agree bit for bit; the others hold the normwise contract
    ex = i0["exact"] & i1["exact"]
    assert ex.mean() > 0.99
    assert np.array_equal(bits(y1[ex]), bits(y0[ex]))
    g, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert O.normwise_ok(y1[~i1["exact"]], g[~i1["exact"]], absdot[~i1["exact"]], 1e-10).all()
    dev = torch.device("cuda", 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    B = torch.from_numpy(np.ascontiguousarray(x.reshape(k, A.ncols).T)).to(dev)
    Cd = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
    for _ in range(3):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    mf.close()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y1))
