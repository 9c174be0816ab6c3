"""GPU parity of the v8 inspector policies at the sizes that trigger them.

* 128-byte K panels for low-similarity rows whose span holds 4-12 L2s of 256-B B rows: the plan must pick 16-column
  fp64 panels, and the output must be BIT-IDENTICAL to the 32-column plan (panels only choose which columns a launch
  computes; every C entry is the same left-to-right FMA chain) and to the oracle on a row sample.
* Tiny-row column windows (K = 1): the plan must chain the row through a few 4 MB windows, bit-identical to the
  unwindowed plan (the chained accumulator restarts from the exact stored value) and to the oracle on a row sample.
Reference kernel: compute_csr, benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:70-96.
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


def run_device(torch, S, A, k, monkeypatch, **envs):
    for name, v in envs.items():
        monkeypatch.setenv(name, str(v))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
    C = torch.full((A.m, k), float("nan"), device=dev, dtype=torch.float64)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    inf, ex = mf.info(), mf.exact_rows()
    mf.close()
    for name in envs:
        monkeypatch.delenv(name)
    return B.cpu().numpy(), C.cpu().numpy(), inf, ex


def sample_rows_exact(O, A, B, C, ex, n=2000, seed=1):
    """Oracle on a row sample (sub-CSR of the sampled rows, B rows gathered): exact rows bit for bit."""
    rng = np.random.default_rng(seed)
    rows = np.sort(rng.choice(A.m, min(n, A.m), replace=False))
    rows = rows[ex[rows].astype(bool)]
    deg = np.diff(A.row_ptr)[rows]
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    cols = np.concatenate([A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows])
    vals = np.concatenate([A.values[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows])
    uc, inv = np.unique(cols, return_inverse=True)
    k = B.shape[1]
    x = np.ascontiguousarray(B[uc].T).reshape(-1)          # column-major [k][len(uc)]
    want = O.spmm(rp, inv.astype(np.int32), vals, len(uc), x, k)
    assert np.array_equal(C[rows].view(np.int64), want.view(np.int64))
    return len(rows)


def test_narrow_panels_bitwise(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params("388875 388875 50 16.6667 normal random 0.3 0 0.5 0.05 14"))
    B, C16, inf16, ex = run_device(torch, S, A, 32, monkeypatch)
    assert inf16[10] == 16 and inf16[11] == 2, inf16        # 128-byte panels chosen by the policy
    _, C32, inf32, _ = run_device(torch, S, A, 32, monkeypatch, SPMM_HIP_PANEL_K=32)
    assert inf32[10] == 32 and inf32[11] == 1
    assert np.array_equal(C16.view(np.int64), C32.view(np.int64))
    assert sample_rows_exact(O, A, B, C16, ex) > 1000


def test_tiny_row_windows_bitwise(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params("1375181 1375181 20 6.6667 normal random 0.6 0 0.5 0.05 14"))
    B, Cw, infw, ex = run_device(torch, S, A, 1, monkeypatch)
    assert 1 < infw[12] <= 12, infw                          # a few chained column windows
    _, C0, inf0, _ = run_device(torch, S, A, 1, monkeypatch, SPMM_HIP_WIN_BYTES=-1)
    assert inf0[12] == 1
    assert np.array_equal(Cw.view(np.int64), C0.view(np.int64))
    assert sample_rows_exact(O, A, B, Cw, ex) > 1000


# Small matrices: narrower K panels of the row kernel, all in ONE launch (blockIdx.y = panel).  Every
# C entry is still the same chain for exact rows (panels only choose which columns a block computes), so the output
# must equal the one-panel plan on every row both plans compute exactly, and be within 1e-10 normwise elsewhere
# (vector lanes / split rows; the separate combine kernel sums the split rows of every panel).
SMALL = ["698 698 500 166.6667 normal random 0.05 0 0.05 0.5 14",          # 4-row blocks, vector lanes
         "65535 65535 5 1.6667 normal random 0.3 0 0.5 0.05 14",           # many short rows
         "3483 3483 100 33.3333 normal random 0.6 1000 0.95 0.95 14"]      # a skewed row: split, combined


@pytest.mark.parametrize("line", SMALL)
@pytest.mark.parametrize("kw", [8, 16])
@pytest.mark.parametrize("k", [32, 128])
def test_small_matrix_one_launch_panels(env, monkeypatch, line, kw, k):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    B0, C0, inf0, ex0 = run_device(torch, S, A, k, monkeypatch, SPMM_HIP_SMALL_KW=0)
    B1, C1, inf1, ex1 = run_device(torch, S, A, k, monkeypatch, SPMM_HIP_SMALL_KW=kw)
    assert np.array_equal(B0, B1)
    assert inf1[10] == kw and inf1[11] == k // kw
    assert np.isfinite(C1).all()
    both = ex0 & ex1
    assert np.array_equal(C1[both].view(np.int64), C0[both].view(np.int64))
    x = np.ascontiguousarray(B0.T).ravel()
    g, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert O.normwise_ok(C1, g, absdot, 1e-10).all()
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(C1[ex1].view(np.int64), seq[ex1].view(np.int64))
