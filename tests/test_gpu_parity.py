"""GPU parity: the HIP engine (through its C ABI) against the oracle and the reference's golden vectors.

Bar: indexing bit-exact; every row the engine reports exact (spmm_hip_exact_rows: rows of <= T
nonzeros, T = the handle's split length, 64..2048, that were not given vector lanes) is one left-to-right FMA chain,
so it must equal the reference kernel BIT FOR BIT (fp64 and fp32); the other rows (split rows, vector lanes) must
be deterministic and satisfy the normwise criterion |C - gold| <= TOL * max(|gold|, sum_j |a_ij b_jn|), TOL = 1e-10 (fp64) / n * 2^-23
(fp32, n = row length), and be identical run to run.  At full size (config 2: 1M x 1M, 20M nnz) parity is checked on a row sample plus size-independent
properties (determinism, linearity in B, layout equivalence).
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
TOL_F64, TOL_F32 = 1e-10, 1e-6


@pytest.fixture(scope="module")
def env():
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    assert S.device_count() >= 1
    return torch, S, O


def gpu_spmm(S, A_rp, A_ci, vals, m, n, x_colmajor, k, want_exact=False):
    mf = S.csr_to_format(A_rp, A_ci, vals, m, n, len(A_ci), k, 0)
    y = np.full(m * k, np.nan, vals.dtype)          # garbage in: every entry must be written
    mf.spmm(np.ascontiguousarray(x_colmajor, vals.dtype), y, k)
    ex = mf.exact_rows()
    assert ex[np.diff(A_rp) > mf.seq_max].sum() == 0     # split rows are never reported exact
    mf.close()
    return (y.reshape(m, k), ex) if want_exact else y.reshape(m, k)


def check_split_aware(O, A_rp, A_ci, vals, ncols, x, k, y, exact, tol):
    """Exact rows bit-exact vs the oracle; the rest normwise vs the Kahan gold."""
    seq = O.spmm(A_rp, A_ci, vals, ncols, x, k)
    short = exact
    assert bits_equal(y[short], seq[short])
    if (~short).any():
        g, absdot = O.gold(A_rp, A_ci, vals.astype(np.float64), ncols, x.astype(np.float64), k)
        assert O.normwise_ok(y[~short], g[~short], absdot[~short], tol).all()


def bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    it = np.int64 if a.dtype == np.float64 else np.int32
    return a.shape == b.shape and np.array_equal(a.view(it), b.view(it))


def _cases(d):
    return sorted({k.split(".")[0] for k in d.files})


def test_golden_spmm_cases_bitwise(env, golden):
    torch, S, O = env
    d = golden("spmm_cases.npz")
    n = 0
    for c in _cases(d):
        rp, ci, va = d[f"{c}.row_ptr"], d[f"{c}.col_idx"], d[f"{c}.vals"]
        m, ncols = (int(v) for v in d[f"{c}.shape"])
        for k in (1, 8, 32, 128):
            if f"{c}.x.k{k}" not in d.files:
                continue
            x = d[f"{c}.x.k{k}"]
            y, short = gpu_spmm(S, rp, ci, va, m, ncols, x, k, want_exact=True)
            assert bits_equal(y[short], d[f"{c}.y_d.k{k}"][short]), (c, k)
            check_split_aware(O, rp, ci, va, ncols, x, k, y, short, TOL_F64)
            yf, short = gpu_spmm(S, rp, ci, va.astype(np.float32), m, ncols, x.astype(np.float32), k, want_exact=True)
            assert bits_equal(yf[short], d[f"{c}.y_f.k{k}"][short]), (c, k, "f32")
            n += 1
    assert n >= 15


def test_golden_mtx_through_gpu(env, golden):
    torch, S, O = env
    d = golden("mtx_csr.npz")
    for c in _cases(d):
        A, _, _ = S.mtx_read(GOLDEN / "mtx" / f"{c}.mtx")
        for k in (1, 4, 32):
            for b in ("ones", "drand48"):
                x = np.ones(A.ncols * k) if b == "ones" else O.drand48(42, A.ncols * k)
                y = gpu_spmm(S, A.row_ptr, A.col_idx, A.values, A.m, A.ncols, x, k)   # rows here are <= 16 nnz
                want = d[f"{c}.y.k{k}.{b}"]
                # duplicates too: the reader restates the reference's (one-thread) duplicate order
                assert bits_equal(y, want), (c, k, b)


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 16, 24, 32, 33, 64, 100, 128, 256])
def test_generated_bitwise_all_k(env, k):
    torch, S, O = env
    A = S.generate(S.gen_params("30000 24000 20 6.6667 normal random 0.3 50 0.95 0.5 14"))
    x = O.drand48(7 + k, A.ncols * k)
    y, ex = gpu_spmm(S, A.row_ptr, A.col_idx, A.values, A.m, A.ncols, x, k, want_exact=True)
    check_split_aware(O, A.row_ptr, A.col_idx, A.values, A.ncols, x, k, y, ex, TOL_F64)
    vf, xf = A.values.astype(np.float32), x.astype(np.float32)
    yf, short = gpu_spmm(S, A.row_ptr, A.col_idx, vf, A.m, A.ncols, xf, k, want_exact=True)
    seqf = O.spmm(A.row_ptr, A.col_idx, vf, A.ncols, xf, k)
    assert bits_equal(yf[short], seqf[short])


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_long_rows_split_path(env, dtype):
    torch, S, O = env
    # skew 2000 at avg 10 -> one row of 20010 nonzeros (> 2048, split whatever T is)
    A = S.generate(S.gen_params("20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.5 3"))
    k = 32
    x = O.drand48(5, A.ncols * k)
    vals = A.values if dtype == "f64" else A.values.astype(np.float32)
    xx = x if dtype == "f64" else x.astype(np.float32)
    y1, ex = gpu_spmm(S, A.row_ptr, A.col_idx, vals, A.m, A.ncols, xx, k, want_exact=True)
    y2 = gpu_spmm(S, A.row_ptr, A.col_idx, vals, A.m, A.ncols, xx, k)
    assert bits_equal(y1, y2), "long-row combine must be deterministic"
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, xx, k)
    deg = np.diff(A.row_ptr)
    long_rows = ~ex
    assert long_rows.sum() >= 1
    assert bits_equal(y1[~long_rows], seq[~long_rows])
    # gold of the inputs the kernel actually saw (fp32-rounded for f32), so only summation error remains
    g, absdot = O.gold(A.row_ptr, A.col_idx, vals.astype(np.float64), A.ncols, xx.astype(np.float64), k)
    if dtype == "f64":
        assert O.normwise_ok(y1, g, absdot, TOL_F64).all()
    else:   # fp32: any-order summation bound gamma_n ~ n * 2^-24 per row (products exact in the fp64 gold + 1 rounding)
        tol = (np.maximum(deg, 1)[:, None] + 1) * 2.0 ** -24 * 1.01
        err = np.abs(y1.astype(np.float64) - g)
        assert (err <= tol * np.maximum(np.abs(g), absdot)).all()


def test_device_layouts_and_host_path_agree(env):
    torch, S, O = env
    A = S.generate(S.gen_params("50000 50000 20 6.6667 normal random 0.3 100 0.95 0.5 14"))
    k = 32
    x = O.drand48(42, A.ncols * k)
    dev = torch.device("cuda", 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    y = np.zeros(A.m * k)
    mf.spmm(x, y, k)
    s = torch.cuda.current_stream().cuda_stream
    Xc = torch.from_numpy(x).to(dev)                                 # column-major [k][ncols]
    Br = torch.from_numpy(x.reshape(k, A.ncols).T.copy()).to(dev)    # row-major [ncols][k]
    C1 = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    C2 = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    mf.statistics_start()                                             # run_device records timing events from here
    mf.spmm_device(Xc.data_ptr(), S.B_COL_MAJOR, C1.data_ptr(), k, s)
    mf.spmm_device(Br.data_ptr(), S.B_ROW_MAJOR, C2.data_ptr(), k, s)
    torch.cuda.synchronize()
    assert bits_equal(C1.cpu().numpy(), y.reshape(A.m, k))
    assert bits_equal(C2.cpu().numpy(), y.reshape(A.m, k))
    t = mf.last_times()
    assert t["kernel_ms"] > 0
    stats = mf.statistics_print_data()
    assert stats.startswith(",") and len(stats.split(",")) == len(S.statistics_print_labels().split(","))
    mf.close()


def test_empty_rows_and_zero_nnz(env):
    torch, S, O = env
    m, n, k = 1000, 300, 8
    rp = np.zeros(m + 1, np.int32)
    y = gpu_spmm(S, rp, np.zeros(0, np.int32), np.zeros(0), m, n, np.ones(n * k), k)
    assert (y == 0).all()
    # mostly-empty matrix with a few rows
    rp[501:] = 3
    ci = np.array([0, 5, 299], np.int32)
    y = gpu_spmm(S, rp, ci, np.array([1.0, 2.0, 3.0]), m, n, np.ones(n * k), k)
    assert (y[500] == 6.0).all() and (np.delete(y, 500, axis=0) == 0).all()


def test_malformed_csr_rejected(env):
    torch, S, O = env
    with pytest.raises(S.SpmmHipError):
        S.csr_to_format(np.array([0, 2], np.int32), np.array([0, 9], np.int32), np.ones(2), 1, 5, 2, 4, 0)
    with pytest.raises(S.SpmmHipError):
        S.csr_to_format(np.array([0, 2, 1], np.int32), np.array([0, 1], np.int32), np.ones(2), 2, 5, 2, 4, 0)


def test_row_shards_equal_whole(env, monkeypatch):
    """Row shards (the multi-GPU split) reproduce the whole matrix: bitwise under a common split length T; under
    the per-handle policy T (which depends on the shard's size) rows <= both T's bitwise, split rows normwise."""
    torch, S, O = env
    p = S.gen_params("40000 40000 20 6.6667 normal random 0.3 100 0.95 0.5 14")
    A = S.generate(p)
    k = 16
    x = O.drand48(1, A.ncols * k)

    def run_all():
        whole, tw = gpu_spmm(S, A.row_ptr, A.col_idx, A.values, A.m, A.ncols, x, k, want_exact=True)
        parts, ts = [], []
        for w in range(3):
            r0, r1 = S.partition_rows(A.row_ptr, A.nnz, 3, w)
            sh = S.generate_rows(p, r0, r1)
            y, t = gpu_spmm(S, sh.row_ptr, sh.col_idx, sh.values, sh.m, A.ncols, x, k, want_exact=True)
            parts.append(y)
            ts.append(t)
        return whole, np.concatenate(parts), tw & np.concatenate(ts)

    whole, parts, short = run_all()
    assert bits_equal(parts[short], whole[short])
    g, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert O.normwise_ok(parts, g, absdot, TOL_F64).all()
    monkeypatch.setenv("SPMM_HIP_SEQ_MAX", "2048")
    monkeypatch.setenv("SPMM_HIP_LANES", "-1")
    whole, parts, short = run_all()
    assert short.all()
    assert bits_equal(parts, whole)


def test_full_size_config2_properties(env):
    """BASELINE config 2 at full size: sampled-row parity, determinism, linearity."""
    torch, S, O = env
    A = S.generate(S.gen_params("1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"))
    k = 32
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    B1 = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
    B2 = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    C1 = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    C1b = torch.empty_like(C1)
    C2 = torch.empty_like(C1)
    C12 = torch.empty_like(C1)
    B12 = B1 + B2
    for B, C in ((B1, C1), (B1, C1b), (B2, C2), (B12, C12)):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, s)
    torch.cuda.synchronize()
    assert torch.equal(C1, C1b)                                         # determinism
    lin = (C12 - (C1 + C2)).abs() <= 1e-13 * (C12.abs() + 1.0)          # linearity (rounding only)
    assert bool(lin.all())
    # sampled rows vs the oracle, bit for bit
    rng = np.random.default_rng(0)
    rows = np.sort(rng.choice(A.m, 3000, replace=False))
    rows = np.union1d(rows, [int(np.argmax(np.diff(A.row_ptr)))])     # include the longest row
    sub_rp = np.zeros(len(rows) + 1, np.int32)
    sub_rp[1:] = np.cumsum(np.diff(A.row_ptr)[rows])
    sub_ci = np.concatenate([A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows])
    sub_va = np.concatenate([A.values[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows])
    x_col = np.ascontiguousarray(B1.cpu().numpy().T).ravel()
    want = O.spmm(sub_rp, sub_ci, sub_va, A.ncols, x_col, k)
    got = C1.cpu().numpy()[rows]
    short = mf.exact_rows()[rows]
    assert bits_equal(got[short], want[short])
    g, absdot = O.gold(sub_rp, sub_ci, sub_va, A.ncols, x_col, k)
    assert O.normwise_ok(got, g, absdot, TOL_F64).all()
    mf.close()


def test_harness_executable_on_mtx(env):
    torch, S, O = env
    exe = ROOT / "spmm-research_amd" / "bin" / "spmm_csr_hip_d.exe"
    envv = dict(os.environ, NUM_COLS="32", USE_ARTIFICIAL_MATRICES="0", SPMM_WARMUP="3", SPMM_TIMED_LOOPS="5",
                SPMM_B_RANDOM="1")
    r = subprocess.run([str(exe), str(GOLDEN / "mtx" / "general_real.mtx")], capture_output=True, text=True,
                       env=envv, timeout=120)
    assert r.returncode == 0, r.stderr
    row = r.stderr.strip().splitlines()[-1].split(",")
    assert row[0].endswith("general_real.mtx") and row[2] == "32" and row[5] == "17"
    assert "errors spmv:" in r.stdout and "Test failed" not in r.stdout
    assert "failing entries=0" in r.stdout
    # synthetic path, one quoted generator line (reference run.sh passes it as one argv)
    envv["USE_ARTIFICIAL_MATRICES"] = "1"
    envv["SPMM_CHECK"] = "1"
    r = subprocess.run([str(exe), "20000 20000 10 3.3333 normal random 0.3 0 0.5 0.5 14"], capture_output=True,
                       text=True, env=envv, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stderr.strip().splitlines()[-1].startswith("synthetic,normal,random,14,20000,20000,")
    assert "failing entries=0" in r.stdout


def test_dlmc_smtx_unsorted_rows(env, tmp_path):
    """DLMC input (USE_DLCM_MATRICES): the CSR is used as stored, so rows may be unsorted and hold duplicates;
    the engine must still follow CSR order bit for bit (windows are never used on unsorted rows), and the harness
    must read the .smtx and pass its accuracy check (negative values: the normwise criterion)."""
    torch, S, O = env
    rng = np.random.default_rng(11)
    m, n = 3000, 2500
    deg = rng.integers(0, 60, m)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = rng.integers(0, n, int(rp[-1])).astype(np.int32)
    f = tmp_path / "dlmc.smtx"
    f.write_text(f"{m}, {n}, {len(ci)}\n" + " ".join(map(str, rp)) + "\n" + " ".join(map(str, ci)) + "\n")
    A = S.smtx_read(f)
    for k in (1, 32):
        x = O.drand48(5 + k, n * k)
        y, ex = gpu_spmm(S, A.row_ptr, A.col_idx, A.values, m, n, x, k, want_exact=True)
        check_split_aware(O, A.row_ptr, A.col_idx, A.values, n, x, k, y, ex, TOL_F64)
    exe = ROOT / "spmm-research_amd" / "bin" / "spmm_csr_hip_d.exe"
    envv = dict(os.environ, NUM_COLS="32", USE_ARTIFICIAL_MATRICES="0", USE_DLCM_MATRICES="1", SPMM_WARMUP="3",
                SPMM_TIMED_LOOPS="5", SPMM_B_RANDOM="1")
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, env=envv, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "failing entries=0" in r.stdout
