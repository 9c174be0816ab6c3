"""Pin the CPU oracle (oracle/spmm_oracle.c) against golden vectors produced by the reference itself
(tests/golden/make_golden.py ran the reference's compiled sources).  CPU only."""
import numpy as np
import pytest

from oracle import oracle as O
from conftest import GOLDEN


def _cases(d):
    return sorted({k.split(".")[0] for k in d.files})


def test_spmm_cases_bitwise_fp64_fp32(golden):
    d = golden("spmm_cases.npz")
    n_checked = 0
    for c in _cases(d):
        rp, ci, va = d[f"{c}.row_ptr"], d[f"{c}.col_idx"], d[f"{c}.vals"]
        m, n = (int(v) for v in d[f"{c}.shape"])
        for k in (1, 8, 32, 128):
            if f"{c}.x.k{k}" not in d.files:
                continue
            x = d[f"{c}.x.k{k}"]
            y = O.spmm(rp, ci, va, n, x, k)
            assert np.array_equal(y.view(np.int64), d[f"{c}.y_d.k{k}"].view(np.int64)), (c, k)
            yf = O.spmm(rp, ci, va.astype(np.float32), n, x.astype(np.float32), k)
            assert np.array_equal(yf.view(np.int32), d[f"{c}.y_f.k{k}"].view(np.int32)), (c, k)
            n_checked += 1
    assert n_checked >= 15


def test_spmm_mtx_fixtures_bitwise(golden):
    d = golden("mtx_csr.npz")
    for c in _cases(d):
        rp, ci, va = d[f"{c}.row_ptr"], d[f"{c}.col_idx"], d[f"{c}.vals"]
        m, n = (int(v) for v in d[f"{c}.shape"])
        for k in (1, 4, 32):
            for b in ("ones", "drand48"):
                x = np.ones(n * k) if b == "ones" else O.drand48(42, n * k)
                y = O.spmm(rp, ci, va, n, x, k)
                assert np.array_equal(y.view(np.int64), d[f"{c}.y.k{k}.{b}"].view(np.int64)), (c, k, b)


def test_spmm_mtx_fixtures_f32_bitwise(golden):
    """fp32 pin: the C restatement on the float build's CSR == the reference FLOAT plugin's output; and the engine's
    host reader (double values, cast to float as the fp32 drivers do) hands the same floats over."""
    import spmm_amd as S
    d = golden("mtx_csr_f32.npz")
    n_checked = 0
    for c in _cases(d):
        rp, ci, va = d[f"{c}.row_ptr"], d[f"{c}.col_idx"], d[f"{c}.vals"]
        assert va.dtype == np.float32
        m, n = (int(v) for v in d[f"{c}.shape"])
        A, _, _ = S.mtx_read(GOLDEN / "mtx" / f"{c}.mtx")
        assert np.array_equal(A.row_ptr, rp) and np.array_equal(A.col_idx, ci), c
        assert np.array_equal(A.values.astype(np.float32).view(np.int32), va.view(np.int32)), c
        for k in (1, 4, 32):
            x = O.drand48(42, n * k).astype(np.float32)
            y = O.spmm(rp, ci, va, n, x, k)
            assert np.array_equal(y.view(np.int32), d[f"{c}.y.k{k}.drand48"].view(np.int32)), (c, k)
            n_checked += 1
    assert n_checked >= 30


def test_partition_matches_reference(golden):
    d = golden("partition.npz")
    for c in _cases(d):
        rp = d[f"{c}.row_ptr"]
        nnz = int(rp[-1])
        for W in (1, 2, 3, 7, 8, 64, 256):
            want = d[f"{c}.W{W}"]
            got = np.array([O.partition(rp, nnz, W, w) for w in range(W)])
            assert np.array_equal(got, want), (c, W)


def test_metrics_match_reference(golden):
    d = golden("metrics.npz")
    for c in _cases(d):
        g, t, want = d[f"{c}.gold"], d[f"{c}.test"], d[f"{c}.metrics"]
        # restated CheckAccuracy over the same (gold, test) pair: gold given in double here
        rp = np.arange(len(g) + 1, dtype=np.int32)
        ci = np.zeros(len(g), np.int32)
        out = O.check_accuracy(rp, ci, g.copy(), 1, np.ones(1), 1, t, 1e-10)
        # the reference sums with OpenMP reductions: compare with a relative tolerance
        np.testing.assert_allclose(out[1:], want, rtol=1e-9, atol=1e-300, err_msg=c)


def test_drand48_stream():
    # POSIX drand48 after srand48(42): first values (glibc)
    v = O.drand48(42, 3)
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.srand48(42)
    libc.drand48.restype = ctypes.c_double
    assert np.array_equal(v, np.array([libc.drand48() for _ in range(3)]))


def test_coo_to_csr_indexing_matches_reference(golden):
    d = golden("mtx_csr.npz")
    # rebuild COO from the reference CSR, shuffle it, and convert back: indexing must be identical
    rng = np.random.default_rng(0)
    for c in _cases(d):
        rp, ci, va = d[f"{c}.row_ptr"], d[f"{c}.col_idx"], d[f"{c}.vals"]
        m = len(rp) - 1
        R = np.repeat(np.arange(m, dtype=np.int32), np.diff(rp))
        perm = rng.permutation(len(R))
        n = int(d[f"{c}.shape"][1])
        rp2, ci2, va2 = O.coo_to_csr(R[perm], ci[perm], va[perm], m, n)
        assert np.array_equal(rp2, rp) and np.array_equal(ci2, ci), c


@pytest.mark.skipif(not O.ref_available("d"), reason="oracle/_ref not built")
def test_restatement_equals_reference_random():
    rng = np.random.default_rng(11)
    m, n = 700, 900
    deg = rng.integers(0, 60, m)
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum(deg)
    ci = np.concatenate([np.sort(rng.choice(n, k, replace=False)) for k in deg]).astype(np.int32)
    va = rng.normal(size=int(rp[-1]))
    for k in (1, 3, 32):
        x = rng.normal(size=n * k)
        assert np.array_equal(O.spmm(rp, ci, va, n, x, k), O.ref_spmm(rp, ci, va.copy(), n, x.copy(), k))
