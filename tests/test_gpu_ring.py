"""GPU parity of the streamed rows (round 6; spmm_kernels.hpp spmm_ring_kernel).

Every row group owns one virtual row and streams its col_idx / values through an LDS slice chunk by chunk; the gathers
and FMAs are the row kernel's, so every row is still ONE fused multiply-add chain from 0 in CSR order.  Forced
streaming (SPMM_HIP_RING=1) must therefore give output BIT-IDENTICAL to the row kernel with every row one chain
(SPMM_HIP_RING=-1, SPMM_HIP_LANES=-1), and the rows reported exact bit-identical to the oracle (reference compute_csr,
spmm_kernel_csr.cpp:70-96): rows of 0 nonzeros, rows shorter than a chunk, rows spanning many chunks with every
start offset modulo 4, split rows (partial slots + the separate combine), lanes past K (K not a power of two), the
last row of the array ending at nnz (the clamped chunk loads), fp64 and fp32, HBM-resident and host-buffer runs.
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


def run(S, A, vals, x, k, ring, monkeypatch, extra=None):
    monkeypatch.setenv("SPMM_HIP_RING", str(ring))
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


MATS = {"avg500": "6000 6000 500 166.6667 normal random 0.3 0 0.5 0.05 14",
        "avg500_band": "4000 4000 500 166.6667 normal random 0.05 100 0.95 0.95 14",
        "avg100_skew": "20000 20000 100 33.3333 normal random 0.3 1000 0.5 0.05 14",   # a giant row: split + combine
        "ragged": "9000 7000 60 60 normal random 0.6 50 0.05 0.05 7"}


RING_CASES = [(k, dt, 1) for k in (8, 32, 40, 128) for dt in ("f64", "f32")] + \
             [(k, dt, mode) for mode in (2, 3) for k in (8, 32, 128) for dt in ("f64", "f32")]


@pytest.mark.parametrize("name", list(MATS))
@pytest.mark.parametrize("k,dtype,mode", RING_CASES)
def test_ring_identical_to_rows_and_oracle(env, monkeypatch, name, k, dtype, mode):
    """mode 1: 16 gathers in flight per row; 2: 32; 3: the software-pipelined row (16 to 32)."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[name]))
    if name == "ragged":
        A = with_empty_rows(S, A, 5)
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")              # every row one chain in the row kernel too
    monkeypatch.setenv("SPMM_HIP_MFMA", "-1")               # no tiles: the row kernel (or the ring) runs every row
    monkeypatch.setenv("SPMM_HIP_TILES", "-1")
    if name != "avg100_skew":
        monkeypatch.setenv("SPMM_HIP_SEQ_MAX", "2048")      # rows stay whole (one chain each): all checked exactly
    x = O.drand48(11 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y0, i0 = run(S, A, vals, xx, k, -1, monkeypatch)
    y1, i1 = run(S, A, vals, xx, k, mode, monkeypatch)
    monkeypatch.setenv("SPMM_HIP_RING", str(mode))
    eligible = k * vals.itemsize >= 64            # row groups of >= 4 sixteen-byte lanes
    assert S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64 if dtype == "f64" else S.F32)["ring"] == \
        (mode if eligible else 0)
    assert np.array_equal(i0["exact"], i1["exact"])
    assert np.array_equal(bits(y1), bits(y0))
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    ex = i1["exact"]
    assert ex.mean() > 0.99
    assert np.array_equal(bits(y1[ex]), bits(seq[ex]))
    if name == "ragged":
        empty = np.diff(A.row_ptr) == 0
        assert empty.sum() > 0 and (bits(y1[empty]) == 0).all()
    if name == "avg100_skew":
        assert i1["split"] >= 1
    if name == "avg100_skew" and dtype == "f64":
        g, absdot = O.gold(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
        assert O.normwise_ok(y1[~ex], g[~ex], absdot[~ex], 1e-10).all()


def test_ring_every_offset_and_tail(env, monkeypatch):
    """Rows of every length 0..300 in order (so row starts take every offset modulo 4 and chunk ends fall everywhere),
    the matrix ending mid-chunk: forced streaming == the row kernel == the oracle, bit for bit."""
    torch, S, O = env
    rng = np.random.default_rng(3)
    lens = np.concatenate([np.arange(301), rng.integers(200, 700, 97)]).astype(np.int64)
    m, ncols = len(lens), 5000
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.concatenate([np.sort(rng.choice(ncols, int(n), replace=False)) for n in lens]).astype(np.int32)
    val = rng.uniform(-1.5, 1.5, int(rp[-1]))
    A = S.CSR(rp, col, val, m, ncols)
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")
    monkeypatch.setenv("SPMM_HIP_MFMA", "-1")
    monkeypatch.setenv("SPMM_HIP_TILES", "-1")
    monkeypatch.setenv("SPMM_HIP_SEQ_MAX", "2048")          # a few hundred rows: keep every row one chain
    for k in (8, 32):
        x = O.drand48(k, ncols * k)
        y0, _ = run(S, A, val, x, k, -1, monkeypatch)
        y1, i1 = run(S, A, val, x, k, 1, monkeypatch)
        assert np.array_equal(bits(y1), bits(y0))
        seq = O.spmm(rp, col, val, ncols, x, k)
        ex = i1["exact"]
        assert ex.all()
        assert np.array_equal(bits(y1), bits(seq))


@pytest.mark.parametrize("k", [32, 128])
def test_ring_device_run(env, monkeypatch, k):
    """HBM-resident runs (spmm_hip_run_device), repeated launches on one handle."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS["avg100_skew"]))
    x = O.drand48(19, A.ncols * k)
    monkeypatch.setenv("SPMM_HIP_MFMA", "-1")
    monkeypatch.setenv("SPMM_HIP_TILES", "-1")
    y_ref, _ = run(S, A, A.values, x, k, 1, monkeypatch)
    dev = torch.device("cuda", 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    B = torch.from_numpy(np.ascontiguousarray(x.reshape(k, A.ncols).T)).to(dev)
    Cd = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
    for _ in range(3):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    mf.close()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y_ref))
