"""GPU: split rows combined inside the row kernel (fused combine) vs the separate combine launch.

The fused path hands partial slots between workgroups (sc1 stores, per-row agent-scope counters, the block whose
add completes a row sums it with sc1 loads and re-arms the counter).  Checked here:
  * it is taken (spmm_hip_info out[18]) whenever a plan has split rows and no column windows;
  * with one K panel it computes the SAME bits as the separate combine kernel (same tree shape);
  * many back-to-back launches on one stream (counters re-armed every launch, uneven load: one row of thousands of
    pieces beside millions of short rows) give identical bits every time;
  * exact rows stay bit-identical to the oracle and split rows satisfy the normwise bound (1e-10 fp64).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_F64 = 1e-10


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


def run_device(torch, S, A, vals, Bt, k, reps=1):
    """reps back-to-back launches into separate C buffers on one stream; returns the list of C (host) and info."""
    dev = torch.device("cuda", 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    mf.plan(k)
    s = torch.cuda.current_stream(dev)
    Cs = [torch.full((A.m, k), float("nan"), dtype=Bt.dtype, device=dev) for _ in range(reps)]
    for C in Cs:
        mf.spmm_device(Bt.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, s.cuda_stream)
    torch.cuda.synchronize()
    info, ex = mf.info(), mf.exact_rows()
    mf.close()
    return [C.cpu().numpy() for C in Cs], info, ex


CASES = [
    # (generator line, forced split length T or None)
    ("20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.5 3", None),     # one 20 K-nonzero row
    ("3000 3000 200 66.6667 normal random 0.3 100 0.5 0.5 5", "64"),      # every row split, many rows per block
    ("200000 200000 8 2.6667 normal random 0.3 30000 0.05 0.5 9", "64"),   # 240 K-nonzero row + 200 K short rows
]


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("k", [1, 8, 32])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_fused_equals_separate_combine(env, monkeypatch, case, k, dtype):
    torch, S, O = env
    line, T = CASES[case]
    if T:
        monkeypatch.setenv("SPMM_HIP_SEQ_MAX", T)
    A = S.generate(S.gen_params(line))
    npd = np.float64 if dtype == "f64" else np.float32
    vals = A.values.astype(npd)
    g = torch.Generator(device="cuda")
    g.manual_seed(11 + k)
    Bt = torch.rand((A.ncols, k), generator=g, device="cuda", dtype=torch.float64 if dtype == "f64" else torch.float32)
    fused, info, ex = run_device(torch, S, A, vals, Bt, k, reps=8)
    assert info[6] > 0 and info[18] == 1, "split rows expected, fused combine expected"
    for C in fused[1:]:
        assert np.array_equal(bits(C), bits(fused[0])), "fused combine must be deterministic launch to launch"
    monkeypatch.setenv("SPMM_HIP_FUSE", "0")
    sep, info0, _ = run_device(torch, S, A, vals, Bt, k)
    assert info0[18] == 0
    if info[11] == 1:    # one K panel: identical tree shape, identical bits
        assert np.array_equal(bits(sep[0]), bits(fused[0])), "fused and separate combine differ"
    x = np.ascontiguousarray(Bt.cpu().numpy().T).ravel()          # column-major for the oracle
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
    assert np.array_equal(bits(fused[0][ex]), bits(seq[ex]))
    if dtype == "f64":
        gd, absdot = O.gold(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
        assert O.normwise_ok(fused[0][~ex], gd[~ex], absdot[~ex], TOL_F64).all()


def test_fused_with_k_panels(env, monkeypatch):
    """K = 128 in 32-column panels: one fused combine per panel launch (counters re-armed between panels)."""
    torch, S, O = env
    monkeypatch.setenv("SPMM_HIP_PANEL_K", "32")
    monkeypatch.setenv("SPMM_HIP_SEQ_MAX", "64")
    A = S.generate(S.gen_params("5000 5000 100 33.3333 normal random 0.3 100 0.5 0.5 21"))
    k = 128
    Bt = torch.rand((A.ncols, k), device="cuda", dtype=torch.float64)
    fused, info, ex = run_device(torch, S, A, A.values, Bt, k, reps=4)
    assert info[11] == 4 and info[18] == 1
    for C in fused[1:]:
        assert np.array_equal(bits(C), bits(fused[0]))
    x = np.ascontiguousarray(Bt.cpu().numpy().T).ravel()
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(bits(fused[0][ex]), bits(seq[ex]))
    gd, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert O.normwise_ok(fused[0], gd, absdot, TOL_F64).all()


def test_fused_graph_replay(env, monkeypatch):
    """The fused path inside a captured hipGraph, replayed many times: bits identical to a plain launch."""
    torch, S, O = env
    monkeypatch.setenv("SPMM_HIP_SEQ_MAX", "64")
    A = S.generate(S.gen_params("50000 50000 20 6.6667 normal random 0.3 1000 0.5 0.5 4"))
    k = 16
    dev = torch.device("cuda", 0)
    Bt = torch.rand((A.ncols, k), device=dev, dtype=torch.float64)
    ref, info, _ = run_device(torch, S, A, A.values, Bt, k)
    assert info[18] == 1
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    mf.plan(k)
    C = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        mf.spmm_device(Bt.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, s.cuda_stream)
    torch.cuda.synchronize()
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph, stream=s):
        for _ in range(4):
            mf.spmm_device(Bt.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    for _ in range(10):
        gph.replay()
    torch.cuda.synchronize()
    assert np.array_equal(bits(C.cpu().numpy()), bits(ref[0]))
    mf.close()
