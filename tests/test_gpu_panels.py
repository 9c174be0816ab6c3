"""Dense panel tiles (spmm_panel_kernel) on the GPU (-m gpu): bit-exact against the row kernel and the
oracle.

A panel row is one left-to-right FMA chain over its nonzeros in CSR order with fma(+0, b, acc) == acc steps between
them (reference compute_csr, spmm_kernel_csr.cpp:70-96), so with panels on every exact row must equal the same row
with panels off (SPMM_HIP_PANELS=-1) bit for bit, and the oracle; B holding inf / NaN must give exactly what the
row kernel gives (the kernel's non-finite fallback); value updates re-gather the panel entries.
"""
import numpy as np
import pytest

from gpu_check import check_rows, sample_rows

pytestmark = pytest.mark.gpu
LINES = ["39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14",     # the verdict's dense band
         "22354 22354 500 166.6667 normal random 0.05 0 0.05 0.05 14",
         "16547 16547 100 33.3333 normal random 0.05 100 0.5 0.5 14",
         "20000 20000 40 13.3333 normal random 0.004 0 0.95 0.5 14"]


@pytest.fixture(scope="module")
def env():
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, S, O


def run(torch, S, A, k, monkeypatch, envs, B=None, dtype=np.float64, vals=None):
    for kk, vv in envs.items():
        monkeypatch.setenv(kk, vv)
    dev = torch.device("cuda", 0)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    if B is None:
        g = torch.Generator(device=dev)
        g.manual_seed(3)
        B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=tdt)
    C = torch.full((A.m, k), float("nan"), device=dev, dtype=tdt)
    v = A.values.astype(dtype) if vals is None else vals
    mf = S.csr_to_format(A.row_ptr, A.col_idx, v, A.m, A.ncols, A.nnz, k, 0)
    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = (C.cpu().numpy(), mf.exact_rows(), mf.panel_info(), mf)
    for kk in envs:
        monkeypatch.delenv(kk)
    return B, out


@pytest.mark.parametrize("line", LINES, ids=["39120x500", "22354x500", "16547x100", "band40"])
def test_panels_bitexact_vs_row_kernel_and_oracle(env, monkeypatch, line):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    k = 32
    B, (c1, ex1, pi1, mf1) = run(torch, S, A, k, monkeypatch, {"SPMM_HIP_PANELS": "1", "SPMM_HIP_PANEL_DENSITY": "0.05"})
    _, (c0, ex0, pi0, mf0) = run(torch, S, A, k, monkeypatch, {"SPMM_HIP_PANELS": "-1"}, B=B)
    mf1.close(), mf0.close()
    assert pi1["tiles"] > 0 and pi1["rows"] > 0.5 * A.m and pi0["tiles"] == 0
    both = ex1 & ex0
    assert ex1.mean() > 0.99 and both.mean() > 0.99
    assert np.array_equal(c1[both].view(np.int64), c0[both].view(np.int64))
    assert np.isfinite(c1).all()
    check_rows(O, A, B.cpu().numpy(), c1, ex1, sample_rows(A, 1500))


def test_panels_fp32_k64_and_k128_panelled(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params(LINES[1]))
    # fp32, K=64: 256-byte B rows
    B, (c1, ex1, pi1, mf) = run(torch, S, A, 64, monkeypatch, {"SPMM_HIP_PANELS": "1"}, dtype=np.float32)
    mf.close()
    assert pi1["tiles"] > 0
    check_rows(O, A, B.cpu().numpy(), c1, ex1, sample_rows(A, 1000), dtype=np.float32)
    # fp64, K=128 cut into 32-column panels: the panel kernel runs once per K panel
    B, (c1, ex1, pi1, mf) = run(torch, S, A, 128, monkeypatch, {"SPMM_HIP_PANELS": "1", "SPMM_HIP_PANEL_K": "32"})
    assert mf.info()[11] == 4 and pi1["tiles"] > 0
    mf.close()
    _, (c0, ex0, _, mf) = run(torch, S, A, 128, monkeypatch, {"SPMM_HIP_PANELS": "-1", "SPMM_HIP_PANEL_K": "32"}, B=B)
    mf.close()
    both = ex1 & ex0
    assert np.array_equal(c1[both].view(np.int64), c0[both].view(np.int64))
    check_rows(O, A, B.cpu().numpy(), c1, ex1, sample_rows(A, 800))


def test_panels_nonfinite_b_fall_back_exactly(env, monkeypatch):
    """inf / NaN in B: a panel's fma(+0, inf) would be NaN where the reference has no product at all -- the kernel
    detects the staged non-finite value and recomputes the tile by the plain chain: same bits as the row kernel."""
    torch, S, O = env
    A = S.generate(S.gen_params(LINES[2]))
    k = 32
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
    B[100, 3] = float("inf")
    B[5000, 7] = float("nan")
    B[5001, :] = -float("inf")
    _, (c1, ex1, pi1, mf1) = run(torch, S, A, k, monkeypatch, {"SPMM_HIP_PANELS": "1", "SPMM_HIP_PANEL_DENSITY": "0.05"}, B=B)
    _, (c0, ex0, _, mf0) = run(torch, S, A, k, monkeypatch, {"SPMM_HIP_PANELS": "-1"}, B=B)
    mf1.close(), mf0.close()
    assert pi1["tiles"] > 0
    both = ex1 & ex0
    nan1, nan0 = np.isnan(c1[both]), np.isnan(c0[both])
    assert nan0.any() and np.array_equal(nan1, nan0)
    assert np.array_equal(c1[both][~nan1].view(np.int64), c0[both][~nan0].view(np.int64))
    # rows that touch none of the poisoned columns are finite in both
    touched = np.zeros(A.m, bool)
    for c in (100, 5000, 5001):
        touched[np.repeat(np.arange(A.m), np.diff(A.row_ptr))[A.col_idx == c]] = True
    assert np.isfinite(c1[~touched]).all()


def test_panels_value_update(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params(LINES[1]))
    k = 32
    B, (c1, ex1, pi1, mf) = run(torch, S, A, k, monkeypatch, {"SPMM_HIP_PANELS": "1"})
    assert pi1["tiles"] > 0
    v2 = (A.values * -0.75 + 0.125).astype(np.float64)
    mf.update_values(v2)
    C = torch.empty((A.m, k), device=B.device, dtype=torch.float64)
    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ex = mf.exact_rows()
    mf.close()
    A2 = S.CSR(A.row_ptr, A.col_idx, v2, A.m, A.ncols)
    check_rows(O, A2, B.cpu().numpy(), C.cpu().numpy(), ex, sample_rows(A, 1500))
