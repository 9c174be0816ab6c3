"""CPU tests of the dense panel decomposition (spmm_hip_debug_panels; kernel spmm_panel_kernel).

A panel tile row must still be ONE left-to-right FMA chain over the row in CSR order (reference compute_csr,
spmm_kernel_csr.cpp:70-96): the kernel walks the tile's union columns in ascending order, so every nonzero of a tile
row must appear exactly once, at the union column equal to its own column, in the chunk holding that column; a row
with a repeated column must stay out of panels (two entries would land on one panel slot); chunks hold <= 32 union
columns; only runs dense enough (nnz / (rows x union) >= the threshold) become tiles.  tests/test_gpu_panels.py then
confirms the kernel bit for bit.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def S():
    import spmm_amd
    return spmm_amd


def band_csr(rng, m, n, per_row, width, dup_rows=()):
    rows = []
    for i in range(m):
        lo = min(max(0, i * n // m - width // 2), n - width)
        c = np.sort(rng.choice(width, per_row, replace=False) + lo)
        if i in dup_rows:
            c = np.sort(np.concatenate([c, c[:2]]))
        rows.append(c)
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    return rp, np.concatenate(rows).astype(np.int32)


def check_panels(S, rp, col, n, min_density=0.15, T=2048):
    t = S.debug_panels(rp, col, n, T, min_density)
    m = len(rp) - 1
    seen = np.zeros(int(rp[-1]), np.int32)
    covered = np.zeros(m, bool)
    ch = t["chunks"]
    for r0, nrows, c0, nc in t["tiles"]:
        assert 1 <= nrows <= 64 and nc >= 1
        assert not covered[r0:r0 + nrows].any()
        covered[r0:r0 + nrows] = True
        union = t["tcol"][ch[c0][0]:ch[c0 + nc][0]]
        assert np.all(np.diff(union) > 0)
        nnz = int(rp[r0 + nrows] - rp[r0])
        assert nnz / (nrows * len(union)) >= min_density - 1e-12
        assert set(union.tolist()) == set(col[rp[r0]:rp[r0 + nrows]].tolist())
        for c in range(c0, c0 + nc):
            x, ncol, e0, ne = ch[c]
            assert 1 <= ncol <= 32 and ch[c + 1][2] == e0 + ne
            cols = t["tcol"][x:x + ncol]
            for e in range(e0, e0 + ne):
                u, r = int(t["pos"][e]) >> 6, int(t["pos"][e]) & 63
                j = int(t["perm"][e])
                assert r < nrows and u < ncol
                assert rp[r0 + r] <= j < rp[r0 + r + 1]              # the entry belongs to row r of the tile
                assert col[j] == cols[u]                            # at its own column
                seen[j] += 1
    assert np.array_equal(covered, t["in_tile"])
    for i in np.flatnonzero(covered):
        assert np.all(seen[rp[i]:rp[i + 1]] == 1)                   # every nonzero of a tile row exactly once
    assert np.all(seen[~np.repeat(covered, np.diff(rp))] == 0)
    return t


def test_dense_band_becomes_panels(S):
    rng = np.random.default_rng(1)
    rp, col = band_csr(rng, 640, 1000, 40, 160)            # 64-row runs: union ~ 260 columns, density ~ 0.35
    t = check_panels(S, rp, col, 1000)
    assert len(t["tiles"]) >= 9 and t["in_tile"].mean() > 0.9


def test_sparse_rows_stay_out(S):
    rng = np.random.default_rng(2)
    rp, col = band_csr(rng, 640, 100000, 20, 50000)        # density ~ 0.0004
    t = check_panels(S, rp, col, 100000)
    assert len(t["tiles"]) == 0 and not t["in_tile"].any()


def test_duplicate_columns_and_long_rows_excluded(S):
    rng = np.random.default_rng(3)
    rp, col = band_csr(rng, 256, 500, 40, 120, dup_rows=(5, 100, 101))
    t = check_panels(S, rp, col, 500)
    assert t["in_tile"].sum() > 200
    for r in (5, 100, 101):
        assert not t["in_tile"][r]
    t = check_panels(S, rp, col, 500, T=30)                 # every row longer than T: no panel
    assert len(t["tiles"]) == 0


def test_threshold_and_halving(S):
    rng = np.random.default_rng(4)
    rp, col = band_csr(rng, 512, 1500, 30, 150)
    lo = check_panels(S, rp, col, 1500, min_density=0.05)
    hi = check_panels(S, rp, col, 1500, min_density=0.5)
    assert lo["in_tile"].sum() > 0 and hi["in_tile"].sum() == 0
    assert lo["in_tile"].sum() >= hi["in_tile"].sum()
