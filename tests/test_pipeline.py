"""CPU tests of the sparse-attention pipeline consumer: the oracle restatement, the mask and weight
generators, and the reference-side plugin build against the reference's pipeline header.

Reference: benchmark_code/CPU/AMD/pipeline_code_bench/ -- compute() step sddmm_bench.cpp:918-937, SDDMM
sddmm_taco_naive.cpp:98-140 (row i of K for every nonzero of row i; the gold at sddmm_bench.cpp:260-276 does the
same), softmax :191-209, mask sddmm_mask.h:16-80,272-294.  The reference plugin needs Intel MKL (absent), so the
restatement is checked against an independent extended-precision computation of the same definitions.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
INTEG = ROOT / "integration"
REF_PIPE_HDR = Path("/root/reference/benchmark_code/CPU/AMD/pipeline_code_bench/sddmm_kernel.h")


@pytest.fixture(scope="module")
def mods():
    from oracle import oracle as O
    from spmm_amd import pipeline as P
    return O, P


def test_mask_generator_band_and_random(mods):
    O, P = mods
    m, band, dens = 300, 6, 0.12
    M = P.band_and_random_mask(m, dens, band, seed=3)
    dense = np.zeros((m, m), bool)
    rows = np.repeat(np.arange(m), np.diff(M.row_ptr))
    dense[rows, M.col_idx] = True
    i, j = np.indices((m, m))
    assert dense[np.abs(i - j) < band].all()                       # the whole band (sddmm_mask.h:53-58)
    extra = dense & ~(np.abs(i - j) < band)
    assert not (extra & (j > i)).any()                              # random entries only where col <= row (:68-69)
    assert M.nnz == int(dens * m * m)                               # placed until density * m^2 (:41,64-75)
    for r in range(m):                                              # dense_to_csr: sorted columns (:272-294)
        assert np.all(np.diff(M.col_idx[M.row_ptr[r]:M.row_ptr[r + 1]]) > 0)
    assert np.all(M.values == 1.0)
    assert np.array_equal(P.band_and_random_mask(m, dens, band, 3).col_idx, M.col_idx)   # seeded


def test_weight_generator(mods):
    O, P = mods
    W = P.dlmc_like_weight(400, 300, 0.25, seed=1)
    assert abs(W.nnz / (400 * 300) - 0.25) < 0.01
    assert W.values.min() >= -1 and W.values.max() < 1
    for r in range(0, 400, 37):
        assert np.all(np.diff(W.col_idx[W.row_ptr[r]:W.row_ptr[r + 1]]) > 0)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_oracle_sddmm_definition(mods, mode, dtype):
    """oracle_sddmm == the definition evaluated in extended precision (within the chain's rounding bound)."""
    O, P = mods
    rng = np.random.default_rng(7)
    m, n = 120, 64
    M = P.band_and_random_mask(m, 0.08, 3, seed=5)
    vals = rng.uniform(0.5, 1.5, M.nnz).astype(dtype)
    Q = rng.uniform(-1, 1, (m, n)).astype(dtype)
    K = rng.uniform(-1, 1, (m, n)).astype(dtype)
    y = O.sddmm(M.row_ptr, M.col_idx, vals, Q, K, mode)
    rows = np.repeat(np.arange(m), np.diff(M.row_ptr))
    kr = M.col_idx if mode else rows
    prod = Q[rows].astype(np.longdouble) * K[kr].astype(np.longdouble)
    want = prod.sum(axis=1) * vals.astype(np.longdouble)
    bound = np.abs(prod).sum(axis=1) * np.abs(vals.astype(np.longdouble)) * (n + 2) * np.finfo(dtype).eps
    assert np.all(np.abs(y.astype(np.longdouble) - want) <= bound)
    if mode == 0:   # the reference's product: every nonzero of a row carries the same chain, scaled by its value
        for r in range(0, m, 11):
            s, e = M.row_ptr[r], M.row_ptr[r + 1]
            assert np.array_equal(y[s:e], (y[s] / vals[s]) * vals[s:e]) or np.allclose(y[s:e] / vals[s:e], y[s] / vals[s])


def test_oracle_softmax(mods):
    O, P = mods
    y = np.random.default_rng(2).normal(0, 3, 5000)
    s = O.softmax(y)
    e = np.exp(y - y.max())
    assert np.allclose(s, e / e.sum(), rtol=1e-12, atol=0)
    assert abs(s.sum() - 1) < 1e-12


def test_oracle_spmm_rowmajor(mods):
    """The row-major entry reuses compute_csr's chain: equal to the column-major call on the transposed x."""
    O, P = mods
    W = P.dlmc_like_weight(90, 70, 0.3, seed=4)
    x = np.random.default_rng(1).uniform(0, 1, (70, 16))
    a = O.spmm_rowmajor(W.row_ptr, W.col_idx, W.values, 70, x)
    b = O.spmm(W.row_ptr, W.col_idx, W.values, 70, np.ascontiguousarray(x.T).ravel(), 16)
    assert np.array_equal(a, b)


@pytest.mark.skipif(not REF_PIPE_HDR.exists(), reason="reference tree absent (the GPU box uses the prebuilt driver)")
def test_pipeline_plugin_builds_against_reference_header():
    r = subprocess.run(["make", "-C", str(INTEG), "-B", str(INTEG / "bin" / "refpipe_driver_d.exe"),
                        str(INTEG / "bin" / "refpipe_driver_f.exe")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "error" not in r.stderr.lower() and "warning" not in r.stderr.lower()
    for vt in ("d", "f"):
        syms = subprocess.run(["nm", "-C", "--defined-only", str(INTEG / "bin" / f"refpipe_driver_{vt}.exe")],
                              capture_output=True, text=True).stdout
        assert "csr_to_format" in syms and "HipPipe::sddmm" in syms and "HipPipe::spmm" in syms
