"""CPU tests of the LDS B tile decomposition (spmm_hip_debug_tiles; kernel spmm_tile_kernel).

A tile row must still be ONE left-to-right FMA chain over the row in CSR order (reference compute_csr,
spmm_kernel_csr.cpp:70-96): chunk by chunk in column order, the row's segments concatenated must be exactly its CSR
range, and every staged column must be the column of the nonzero that reads it (padding entries -- value -0 on
the zero B row -- only at the end of a segment, which is a multiple of 4 entries).  These invariants, plus the LDS
limits the kernel relies on (<= uc columns and <= capa nonzeros per chunk, 8-aligned offsets), are what the GPU
parity tests (tests/test_gpu_tiles.py) then confirm bit for bit.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def S():
    import spmm_amd
    return spmm_amd


def check_tiles(S, rp, col, ncols, T=2048, rmax=64, uc=128, capa=2048, min_reuse=1.0, colmax=0, dmax=0):
    t = S.debug_tiles(rp, col, ncols, T, rmax, uc, capa, min_reuse, colmax, dmax)
    m = len(rp) - 1
    seen = np.zeros(int(rp[-1]), np.int32)
    covered = np.zeros(m, bool)
    ch = t["chunks"]
    for r0, nrows, c0, nc in t["tiles"]:
        assert 1 <= nrows <= rmax and nc >= 1 and (dmax <= 0 or nc <= dmax)
        assert colmax <= 0 or ch[c0 + nc][0] - ch[c0][0] <= colmax
        assert not covered[r0:r0 + nrows].any()
        covered[r0:r0 + nrows] = True
        nxt = rp[r0:r0 + nrows].astype(np.int64).copy()        # next expected nonzero of each row
        prev_last_col = -1
        for c in range(c0, c0 + nc):
            x, ncol, a, w = ch[c]
            a1, w1 = ch[c + 1][2], ch[c + 1][3]
            assert a % 8 == 0 and w % 8 == 0 and 1 <= ncol <= uc
            cols = t["tcol"][x:x + ncol]
            assert np.all(np.diff(cols) > 0) and cols[0] > prev_last_col      # sorted union, chunks in order
            prev_last_col = cols[-1]
            seg = t["tseg"][w:w + nrows + 1].astype(np.int64)
            assert seg[0] == 0 and np.all(np.diff(seg) >= 0) and seg[-1] <= capa and a + seg[-1] <= a1
            assert w1 - w >= nrows + 1
            assert np.all(seg % 4 == 0)                                        # padded segments
            for q in range(nrows):
                pos = np.arange(a + seg[q], a + seg[q + 1])
                real = t["perm"][pos] >= 0
                n = int(real.sum())
                assert np.all(real[:n]) and len(pos) - n < 4                      # padding only at the end
                assert np.all(t["tlidx"][pos[n:]] == 0xFFFF)
                pos = pos[:n]
                js = t["perm"][pos]
                assert np.array_equal(js, np.arange(nxt[q], nxt[q] + n))        # CSR order, contiguous
                assert np.array_equal(cols[t["tlidx"][pos]], col[js])            # staged column == nonzero's
                seen[js] += 1
                nxt[q] += n
            assert np.all(t["perm"][a + seg[-1]:a1] == -1)                     # only padding after the segments
        assert np.array_equal(nxt, rp[r0 + 1:r0 + nrows + 1])                   # every row complete
    assert np.array_equal(t["in_tile"], covered)
    in_rows = np.repeat(covered, np.diff(rp))
    assert np.all(seen[in_rows] == 1) and np.all(seen[~in_rows] == 0)
    return t


@pytest.mark.parametrize("line", ["3000 3000 100 33 normal random 0.05 0 0.95 0.95 14",
                                  "5000 8000 20 6.6667 normal random 0.3 100 0.95 0.5 7",
                                  "2000 2000 300 100 normal random 0.05 10 1.4 0.95 14",
                                  "4000 4000 5 1.6667 normal random 0.6 0 0.05 0.05 14"])
def test_tile_invariants_generated(S, line):
    A = S.generate(S.gen_params(line))
    for uc, capa, colmax, dmax in ((128, 2048, 0, 0), (16, 400, 0, 0), (4096, 2048, 0, 0), (48, 896, 2172, 63),
                                   (48, 896, 300, 8)):
        check_tiles(S, A.row_ptr, A.col_idx, A.ncols, uc=uc, capa=capa, colmax=colmax, dmax=dmax)


def test_tile_reuse_threshold(S):
    """Tiles below the reuse threshold stay with the row kernel; above it they are taken."""
    A = S.generate(S.gen_params("6000 6000 50 16 normal random 0.05 0 0.95 0.95 14"))
    hi = check_tiles(S, A.row_ptr, A.col_idx, A.ncols, min_reuse=4.0)
    assert hi["in_tile"].mean() > 0.9
    B = S.generate(S.gen_params("6000 600000 20 6 normal random 0.6 0 0.05 0.05 14"))   # no shared columns
    lo = check_tiles(S, B.row_ptr, B.col_idx, B.ncols, min_reuse=4.0)
    assert lo["in_tile"].sum() == 0


def test_tile_edge_cases(S):
    rng = np.random.default_rng(3)
    m, n = 300, 50
    lens = rng.integers(0, 12, m)
    lens[5:20] = 0                                                  # empty rows inside a tile
    lens[100] = 3000                                                # a row longer than T: never in a tile
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.concatenate([np.sort(rng.integers(0, n, L)) for L in lens]).astype(np.int32)   # duplicates allowed
    t = check_tiles(S, rp, col, n, T=2048, rmax=64, uc=8, capa=400)
    assert not t["in_tile"][100]
    assert t["in_tile"][5:20].all()
    # one column repeated more often than a chunk can hold: that tile stays with the row kernel
    rp2 = np.array([0, 100, 200], np.int32)
    col2 = np.zeros(200, np.int32)
    t2 = check_tiles(S, rp2, col2, 4, capa=64)
    assert t2["in_tile"].sum() == 0
    # empty matrix / all-empty rows
    t3 = check_tiles(S, np.zeros(11, np.int32), np.zeros(0, np.int32), 5)
    assert t3["in_tile"].sum() == 0


def test_tile_unsorted_rejected(S):
    rp = np.array([0, 3], np.int32)
    with pytest.raises(S.SpmmHipError):
        S.debug_tiles(rp, np.array([2, 1, 0], np.int32), 3, 2048)


def test_tile_index_guard(S, monkeypatch):
    """tile tables use 32-bit positions; a decomposition whose padded tables reach the limit is refused
    (the plan then keeps those rows in the row kernel).  The limit is lowered here so a small matrix reaches it."""
    rng = np.random.default_rng(3)
    m, n = 256, 96
    rows = [np.sort(rng.choice(n, 40, replace=False)) for _ in range(m)]
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    t = S.debug_tiles(rp, col, n, 2048, 32, 48, 896, 1.0)
    nz = len(t["perm"])
    assert nz >= rp[-1]
    monkeypatch.setenv("SPMM_HIP_TILE_INDEX_LIMIT", str(nz))          # padded positions + 64 >= limit: refused
    with pytest.raises(S.SpmmHipError) as e:
        S.debug_tiles(rp, col, n, 2048, 32, 48, 896, 1.0)
    assert e.value.status == -7
    monkeypatch.setenv("SPMM_HIP_TILE_INDEX_LIMIT", str(nz + 4096))   # within the limit: accepted
    assert len(S.debug_tiles(rp, col, n, 2048, 32, 48, 896, 1.0)["perm"]) == nz
