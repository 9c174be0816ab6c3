"""GPU parity of the paired short rows (round 6; spmm_kernels.hpp rows_pair_step).

A row group takes its rows two at a time in one gather batch (row r in the first half of the slots, row r + NG in the
second) when every group of the wave has both rows within half a batch; otherwise the plain per-row loop runs.  Every
row is still ONE fused multiply-add chain from 0 in CSR order, so forced pairing (SPMM_HIP_PAIR=1) must give output
BIT-IDENTICAL to the unpaired kernel (SPMM_HIP_PAIR=-1) on every row, and rows reported exact bit-identical to the
oracle (reference compute_csr, spmm_kernel_csr.cpp:70-96): empty rows, ragged rows (pair and single steps mixed),
rows longer than a batch, split rows (partial slots + the fused and the separate combine), K not a multiple of the
lane width, fp64 and fp32, HBM-resident and host-buffer runs.
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


def run(S, A, vals, x, k, pair, monkeypatch, extra=None):
    monkeypatch.setenv("SPMM_HIP_PAIR", str(pair))
    for kk, vv in (extra or {}).items():
        monkeypatch.setenv(kk, vv)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    out = {"exact": mf.exact_rows(), "split": int(mf.info()[6]), "lmax": int(mf.info()[16])}
    mf.close()
    return y.reshape(A.m, k), out


def with_empty_rows(S, A, every):
    """A copy of A whose every `every`-th row is emptied (rows of 0 nonzeros must store 0)."""
    keep = np.ones(A.nnz, bool)
    for r in range(0, A.m, every):
        keep[A.row_ptr[r]:A.row_ptr[r + 1]] = False
    lens = np.diff(A.row_ptr).copy()
    lens[::every] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    return S.CSR(rp, A.col_idx[keep].copy(), A.values[keep].copy(), A.m, A.ncols)


MATS = {"avg5": "60000 60000 5 1.6667 normal random 0.6 0 0.05 0.05 14",
        "avg5_similar": "60000 60000 5 1.6667 normal random 0.05 0 1.4 0.95 14",
        "avg10_skew": "30000 30000 10 3.3333 normal random 0.3 1000 0.5 0.05 14",   # one long row: split + combine
        "avg20": "20000 20000 20 6.6667 normal random 0.05 0 0.95 0.05 14",         # rows longer than a batch
        "ragged": "40000 30000 6 4 normal random 0.6 50 0.05 0.05 7"}


@pytest.mark.parametrize("name", list(MATS))
@pytest.mark.parametrize("k", [4, 8, 32, 40, 128])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_paired_identical_to_unpaired_and_oracle(env, monkeypatch, name, k, dtype):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[name]))
    if name == "avg5":
        A = with_empty_rows(S, A, 7)
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")              # every row one chain: exact rows checked against the oracle
    x = O.drand48(5 + k, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y0, i0 = run(S, A, vals, xx, k, -1, monkeypatch)
    y1, i1 = run(S, A, vals, xx, k, 1, monkeypatch)
    eligible = k * vals.itemsize >= 32            # row groups of >= 2 lanes (16-byte lanes); one-lane groups never pair
    monkeypatch.setenv("SPMM_HIP_PAIR", "1")
    assert S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64 if dtype == "f64" else S.F32)["pair"] == eligible
    assert np.array_equal(i0["exact"], i1["exact"])
    assert np.array_equal(bits(y1), bits(y0))
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    ex = i1["exact"]
    assert ex.mean() > 0.99
    assert np.array_equal(bits(y1[ex]), bits(seq[ex]))
    if name == "avg5":
        empty = np.diff(A.row_ptr) == 0
        assert empty.sum() > 0 and (bits(y1[empty]) == 0).all()
    if name == "avg10_skew":
        assert i1["split"] >= 1


@pytest.mark.parametrize("k", [8, 32])
def test_paired_device_run_and_separate_combine(env, monkeypatch, k):
    """HBM-resident run (spmm_hip_run_device) and the separate combine launch (SPMM_HIP_FUSE=0) with pairing; default
    lane policy, so the split row's pieces take vector lanes in their own blocks while the other blocks pair."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS["avg10_skew"]))
    x = O.drand48(17, A.ncols * k)
    monkeypatch.delenv("SPMM_HIP_LANES", raising=False)
    y_ref, _ = run(S, A, A.values, x, k, -1, monkeypatch)
    for extra in ({}, {"SPMM_HIP_FUSE": "0"}):
        y1, i1 = run(S, A, A.values, x, k, 1, monkeypatch, extra)
        assert np.array_equal(bits(y1), bits(y_ref))
    monkeypatch.setenv("SPMM_HIP_FUSE", "1")
    monkeypatch.setenv("SPMM_HIP_PAIR", "1")
    dev = torch.device("cuda", 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    B = torch.from_numpy(np.ascontiguousarray(x.reshape(k, A.ncols).T)).to(dev)
    Cd = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
    for _ in range(3):                                         # repeated launches: the combine counters re-arm
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    mf.close()
    assert np.array_equal(bits(Cd.cpu().numpy()), bits(y_ref))


def test_pair_policy_short_rows_only(env, monkeypatch):
    """Policy: fp64 launches of >= 4 M nonzeros whose rows average <= 6 nonzeros and whose 16-row windows share
    columns pair at K 4..32; rows without shared columns, longer rows, smaller matrices, fp32, one-lane row groups
    (K = 1) and 64-lane groups (K = 128) do not."""
    torch, S, O = env
    monkeypatch.delenv("SPMM_HIP_PAIR", raising=False)
    monkeypatch.delenv("SPMM_HIP_LANES", raising=False)
    similar = "1000000 1000000 5 1.6667 normal random 0.6 0 0.05 0.95 14"
    for line, k, dt, want in ((similar, 32, S.F64, True), (similar, 8, S.F64, True), (similar, 1, S.F64, False),
                              (similar, 128, S.F64, False), (similar, 32, S.F32, False),
                              ("400000 400000 5 1.6667 normal random 0.6 0 0.05 0.95 14", 32, S.F64, False),
                              ("1000000 1000000 5 1.6667 normal random 0.6 0 0.05 0.05 14", 32, S.F64, False),
                              ("300000 300000 20 6.6667 normal random 0.6 0 0.05 0.95 14", 32, S.F64, False)):
        A = S.generate(S.gen_params(line))
        p = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, dt)
        assert bool(p["pair"]) == want, (line, k, dt, p["pair_reuse"])
