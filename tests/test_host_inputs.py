"""Product host input path (libspmm_host.so / libspmm_hip.so host-only entry points) against the reference's
golden fixtures.  CPU only: nothing here touches a GPU."""
from pathlib import Path

import numpy as np
import pytest

import spmm_amd as S

GOLDEN = Path(__file__).resolve().parent / "golden"


def _cases(d):
    return sorted({k.split(".")[0] for k in d.files})


def test_mtx_reader_matches_reference_indexing(golden):
    d = golden("mtx_csr.npz")
    for c in _cases(d):
        A, field, sym = S.mtx_read(GOLDEN / "mtx" / f"{c}.mtx")
        m, n = (int(v) for v in d[f"{c}.shape"])
        assert (A.m, A.ncols) == (m, n), c
        assert np.array_equal(A.row_ptr, d[f"{c}.row_ptr"]), c
        assert np.array_equal(A.col_idx, d[f"{c}.col_idx"]), c
        # values bit for bit, duplicates included (the reference's one-thread order, tests/golden/make_golden.py)
        assert np.array_equal(A.values.view(np.int64), d[f"{c}.vals"].view(np.int64)), c


def test_mtx_reader_rejects_malformed(tmp_path):
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\n3 3 2\n1 1 1.0\n")  # one entry short
    with pytest.raises(ValueError):
        S.mtx_read(bad)
    bad.write_text("%%MatrixMarket matrix coordinate real weird\n1 1 1\n1 1 1.0\n")
    with pytest.raises(ValueError):
        S.mtx_read(bad)
    bad.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n")  # row out of range
    with pytest.raises(ValueError):
        S.mtx_read(bad)


def write_smtx(path, rp, ci, m, n):
    """DLMC .smtx text as the reference reader expects it (dlcm_matrix.c:223, dlcm_matrix_gen.c:82-106)."""
    path.write_text(f"{m}, {n}, {len(ci)}\n" + " ".join(map(str, rp)) + "\n" + " ".join(map(str, ci)) + "\n")


def test_smtx_reader_keeps_stored_csr(tmp_path):
    """USE_DLCM_MATRICES path: offsets and columns used exactly as stored (no coo_to_csr, no column sort),
    values a seeded U[-1, 1) stream (the reference seeds from time(NULL), so values are not pinnable)."""
    rng = np.random.default_rng(3)
    m, n = 37, 53
    deg = rng.integers(0, 9, m)
    deg[5] = 0
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    ci = rng.integers(0, n, int(rp[-1])).astype(np.int32)       # unsorted rows, duplicates allowed
    f = tmp_path / "a.smtx"
    write_smtx(f, rp, ci, m, n)
    A = S.smtx_read(f, value_seed=7)
    assert (A.m, A.ncols, A.nnz) == (m, n, int(rp[-1]))
    assert np.array_equal(A.row_ptr, rp) and np.array_equal(A.col_idx, ci)
    assert np.array_equal(A.values, S.uniform(7, -1.0, 1.0, A.nnz))
    assert np.array_equal(S.smtx_read(f, value_seed=7).values, A.values)
    e = tmp_path / "empty.smtx"
    e.write_text("4, 6, 0\n0 0 0 0 0\n")
    E = S.smtx_read(e)
    assert (E.m, E.ncols, E.nnz) == (4, 6, 0) and np.array_equal(E.row_ptr, np.zeros(5, np.int32))


def test_smtx_reader_matches_reference(golden):
    """Pinned against the reference's own smtx_read (dlcm_matrix.c:258-324, compiled into oracle/_ref): the
    offsets and columns it returns for the committed DLMC files (tests/golden/smtx/, make_golden.py).  Values are
    time-seeded in the reference (srand(time(NULL))), so only the structure is pinnable."""
    d = golden("smtx_csr.npz")
    cases = _cases(d)
    assert len(cases) >= 4
    for c in cases:
        A = S.smtx_read(GOLDEN / "smtx" / f"{c}.smtx")
        m, k = (int(v) for v in d[f"{c}.shape"])
        assert (A.m, A.ncols, A.nnz) == (m, k, len(d[f"{c}.col_idx"])), c
        assert np.array_equal(A.row_ptr, d[f"{c}.row_ptr"]), c
        assert np.array_equal(A.col_idx, d[f"{c}.col_idx"]), c


def test_smtx_reader_matches_reference_live(tmp_path):
    """Same pin on fresh random files when oracle/_ref is built (this container only)."""
    import oracle.oracle as O
    if not O.ref_available("d"):
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(11)
    for t in range(6):
        m, n = int(rng.integers(1, 80)), int(rng.integers(1, 90))
        deg = rng.integers(0, 12, m)
        rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
        ci = rng.integers(0, n, int(rp[-1])).astype(np.int32)
        f = tmp_path / f"r{t}.smtx"
        write_smtx(f, rp, ci, m, n)
        rm, rk, rrp, rci = O.ref_smtx_read(str(f))
        A = S.smtx_read(f)
        assert (A.m, A.ncols) == (rm, rk)
        assert np.array_equal(A.row_ptr, rrp) and np.array_equal(A.col_idx, rci)


@pytest.mark.parametrize("text", ["3 3 2\n0 1 2 2\n0 1\n",         # header without commas
                                  "3, 3, 2\n0 1 2\n0 1\n",          # short offsets line
                                  "3, 3, 2\n0 2 1 2\n0 1\n",        # decreasing offsets
                                  "3, 3, 2\n0 1 2 3\n0 1\n",        # last offset != nnz
                                  "3, 3, 2\n0 1 2 2\n0 3\n",        # column out of range
                                  "3, 3, 2\n0 1 2 2\n0\n"])         # short column line
def test_smtx_reader_rejects_malformed(tmp_path, text):
    f = tmp_path / "bad.smtx"
    f.write_text(text)
    with pytest.raises(ValueError):
        S.smtx_read(f)


def test_mtx_array_format(tmp_path):
    f = tmp_path / "dense.mtx"
    f.write_text("%%MatrixMarket matrix array real general\n2 3\n1\n2\n3\n4\n5\n6\n")
    A, field, sym = S.mtx_read(f)
    assert A.m == 2 and A.ncols == 3 and A.nnz == 6
    dense = np.zeros((2, 3))
    for i in range(2):
        for j in range(A.row_ptr[i], A.row_ptr[i + 1]):
            dense[i, A.col_idx[j]] = A.values[j]
    assert np.array_equal(dense, np.array([[1, 3, 5], [2, 4, 6]], float))


def test_coo_to_csr_matches_reference(golden):
    d = golden("mtx_csr.npz")
    rng = np.random.default_rng(5)
    for c in _cases(d):
        rp, ci, va = d[f"{c}.row_ptr"], d[f"{c}.col_idx"], d[f"{c}.vals"]
        m = len(rp) - 1
        R = np.repeat(np.arange(m, dtype=np.int32), np.diff(rp))
        p = rng.permutation(len(R))
        A = S.coo_to_csr(R[p], ci[p], va[p], m)
        assert np.array_equal(A.row_ptr, rp) and np.array_equal(A.col_idx, ci), c


def test_partition_rows_matches_reference(golden):
    d = golden("partition.npz")
    for c in _cases(d):
        rp = d[f"{c}.row_ptr"]
        nnz = int(rp[-1])
        for W in (1, 2, 3, 7, 8, 64, 256):
            got = np.array([S.partition_rows(rp, nnz, W, w) for w in range(W)])
            assert np.array_equal(got, d[f"{c}.W{W}"]), (c, W)


def test_check_accuracy_metrics_match_reference(golden):
    d = golden("metrics.npz")
    for c in _cases(d):
        g, t, want = d[f"{c}.gold"], d[f"{c}.test"], d[f"{c}.metrics"]
        A = S.CSR(np.arange(len(g) + 1, dtype=np.int32), np.zeros(len(g), np.int32), g.copy(), len(g), 1)
        out = S.check_accuracy(A, np.ones(1), 1, t, 1e-10)
        np.testing.assert_allclose(out[1:9], want, rtol=1e-9, atol=1e-300, err_msg=c)


def test_check_accuracy_normwise_cancellation():
    # a row whose exact sum cancels to ~0: pointwise relative error explodes, normwise check stays meaningful
    rp = np.array([0, 2], np.int32)
    ci = np.array([0, 1], np.int32)
    va = np.array([1.0, -1.0])
    A = S.CSR(rp, ci, va, 1, 2)
    x = np.array([1.0, 1.0 + 2**-40])
    y = np.array([1e-16])  # slightly off the exact -2^-40 ... still within eps * sum|ab|
    out = S.check_accuracy(A, x, 1, y, 1e-10)
    assert out[9] == 0.0


def test_generator_deterministic_and_row_ranges():
    p = S.gen_params("30000 25000 12 4 normal random 0.3 50 0.95 0.5 14")
    A = S.generate(p)
    B = S.generate(p)
    assert np.array_equal(A.row_ptr, B.row_ptr) and np.array_equal(A.col_idx, B.col_idx)
    assert np.array_equal(A.values, B.values)
    assert np.array_equal(S.generate_row_ptr(p), A.row_ptr)
    for r0, r1 in ((0, 1), (4095, 4097), (10000, 30000), (29999, 30000)):
        sub = S.generate_rows(p, r0, r1)
        a, b = A.row_ptr[r0], A.row_ptr[r1]
        assert np.array_equal(sub.col_idx, A.col_idx[a:b])
        assert np.array_equal(sub.row_ptr, A.row_ptr[r0:r1 + 1] - a)
    # well-formed CSR: sorted unique columns per row, in range
    assert A.col_idx.min() >= 0 and A.col_idx.max() < A.ncols
    d = np.diff(A.col_idx)
    starts = A.row_ptr[1:-1]
    mask = np.ones(len(d), bool)
    mask[starts[(starts > 0) & (starts < len(A.col_idx))] - 1] = False
    assert (d[mask] > 0).all()
    assert ((A.values >= 0.5) & (A.values < 1.5)).all()


@pytest.mark.parametrize("line,tol", [
    ("200000 200000 20 6.6667 normal random 0.3 100 0.95 0.5 14", None),
    ("100000 100000 10 3.3333 normal random 0.05 0 0.05 0.05 14", None),
    ("100000 100000 20 6.6667 normal random 0.05 1000 1.4 0.75 14", None),
    ("50000 50000 50 16.6667 gamma random 0.3 0 0.5 0.25 14", None),
])
def test_generator_features_near_targets(line, tol):
    p = S.gen_params(line)
    A = S.generate(p)
    f = S.features(A)
    assert abs(f["avg_nnz_per_row"] - p.avg_nnz_per_row) / p.avg_nnz_per_row < 0.02
    if p.skew == 0:  # one giant row dominates the std otherwise
        assert abs(f["std_nnz_per_row"] - p.std_nnz_per_row) / p.std_nnz_per_row < 0.15
    else:
        assert abs(f["skew"] - p.skew) / p.skew < 0.02
    assert abs(f["avg_bw_scaled"] - p.bw) < 0.35 * p.bw + 0.01
    assert abs(f["avg_num_neighbours"] - p.avg_num_neighbours) < 0.25
    assert abs(f["cross_row_similarity"] - p.cross_row_similarity) < 0.15


def test_bytes_alg_model():
    # 4(m+1) + (4+s) nnz + s K ncols + s K m
    assert S.bytes_alg(10, 20, 30, 4, S.F64) == 4 * 11 + 12 * 30 + 8 * 4 * 20 + 8 * 4 * 10
    assert S.bytes_alg(10, 20, 30, 4, S.F32) == 4 * 11 + 8 * 30 + 4 * 4 * 20 + 4 * 4 * 10


def _random_dup_mtx(rng, path, m, n, nnz, col_span):
    R = rng.integers(0, m, nnz)
    C = rng.integers(0, col_span, nnz)
    V = np.arange(1, nnz + 1, dtype=np.float64)          # distinct values: the order of duplicates is visible
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate real general\n{m} {n} {nnz}\n")
        for r, c, v in zip(R, C, V):
            f.write(f"{r + 1} {c + 1} {v}\n")
    return R, C, V


def test_duplicate_order_matches_reference_one_thread(tmp_path):
    """Random COO with many duplicate (row, col) entries through both sorts of csr_sort_columns (rows longer than
    n/5: stable bucket sort; shorter: the reference quicksort): values in the reference's order, bit for bit,
    for the product reader and the oracle, against the reference built from its sources and run with one thread.
    Rows are kept no longer than min(m, n): the reference's sort buffers are sized m and n (csr_gen.c:100-103)."""
    from oracle import oracle as O
    if not O.ref_available("d"):
        pytest.skip("oracle/_ref not built")
    L = O.ref_lib("d")
    L.ref_set_threads(1)
    rng = np.random.default_rng(0)
    done = 0
    for t in range(120):
        m, n = int(rng.integers(60, 120)), int(rng.integers(2, 400))
        nnz = int(rng.integers(0, 600))
        span = max(1, n // int(rng.integers(1, 20)))
        path = tmp_path / f"dup{t}.mtx"
        R, C, V = _random_dup_mtx(rng, path, m, n, nnz, span)
        if nnz and np.bincount(R).max() >= min(m, n):
            continue
        _, _, rp, ci, va = O.ref_mtx_to_csr(str(path), "d")
        A, _, _ = S.mtx_read(path)
        assert np.array_equal(A.row_ptr, rp) and np.array_equal(A.col_idx, ci) and np.array_equal(A.values, va), t
        rp2, ci2, va2 = O.coo_to_csr(R, C, V, m, n)
        assert np.array_equal(rp2, rp) and np.array_equal(ci2, ci) and np.array_equal(va2, va), t
        B = S.coo_to_csr(R, C, V, m, n)
        assert np.array_equal(B.values, va), t
        done += 1
    assert done > 80
