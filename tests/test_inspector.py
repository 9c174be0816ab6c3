"""Inspector work decomposition (host only, spmm_hip_debug_inspect): plain row split and column windows.

Column windows (chained mode, spmm_engine.hip inspect_windows) cut every row (or split-row piece) where its column
window changes; launch w processes window w's segments and a segment that is not its piece's first continues the
FMA chain from the value the previous window stored.  These tests prove on the CPU that the decomposition keeps
the reference's operation order (compute_csr, spmm_kernel_csr.cpp:70-96: one left-to-right chain per row):
every nonzero appears once, a destination's segments concatenated in window order are exactly its CSR range in
order, only the first segment starts from 0, and an emulation of the chained launches gives the same bits as the
unbroken chain.
"""
import numpy as np
import pytest

import spmm_amd as S

CAP_ROWS = 512


def _matrices():
    rng = np.random.default_rng(7)
    out = []
    for line in ("3000 2500 20 6.6667 normal random 0.3 100 0.95 0.5 14",
                 "2000 4000 60 20 normal random 0.05 1000 1.4 0.5 14",
                 "700 700 200 66.6667 normal random 0.6 10 0.5 0.95 14"):
        A = S.generate(S.gen_params(line))
        out.append((line, A.row_ptr, A.col_idx, A.ncols))
    # empty rows, a long row, a row in one column (duplicates), an all-empty tail
    m, n = 300, 1000
    rows = []
    for i in range(m):
        if i % 7 == 0 or i > 280:
            rows.append(np.zeros(0, np.int32))
        elif i == 13:
            rows.append(np.sort(rng.integers(0, n, 5000)).astype(np.int32))
        elif i == 14:
            rows.append(np.full(9, 500, np.int32))
        else:
            rows.append(np.sort(rng.integers(0, n, rng.integers(1, 40))).astype(np.int32))
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    out.append(("handmade", rp, np.concatenate(rows), n))
    return out


MATS = _matrices()


def _pieces(rp, T):
    """{dest: (start, end)} of the row split: rows <= T whole, longer rows in T-nonzero pieces to slots."""
    pcs, slot = {}, 0
    for r in range(len(rp) - 1):
        s, e = int(rp[r]), int(rp[r + 1])
        if e - s <= T:
            pcs[r] = (s, e)
        else:
            for q in range((e - s + T - 1) // T):
                pcs[-(slot + q) - 1] = (s + q * T, min(s + (q + 1) * T, e))
            slot += (e - s + T - 1) // T
    return pcs


def _check_blocks(ins, cap, T):
    vp, blk, wb = ins["vrow_ptr"], ins["blk"], ins["win_blk"]
    for w in range(len(wb) - 1):
        covered = []
        for b in range(wb[w], wb[w + 1]):
            v0, v1 = blk[b]
            assert 0 < v1 - v0 <= CAP_ROWS
            assert vp[v1] - vp[v0] <= max(cap, T)
            covered.append((v0, v1))
        covered.sort()
        for (a0, a1), (b0, b1) in zip(covered, covered[1:]):
            assert a1 == b0
        if covered:
            yield w, covered[0][0], covered[-1][1]


@pytest.mark.parametrize("name,rp,col,ncols", MATS, ids=[m[0][:24] for m in MATS])
@pytest.mark.parametrize("T", [64, 2048])
@pytest.mark.parametrize("wcols", [0, 37, 256, 100000])
def test_decomposition_keeps_csr_order(name, rp, col, ncols, T, wcols):
    cap = 2048
    ins = S.debug_inspect(rp, col, ncols, T, cap, wcols)
    nnz = int(rp[-1])
    vp, vd = ins["vrow_ptr"], ins["vdest"]
    assert vp[0] == 0 and vp[-1] == nnz and np.all(np.diff(vp) >= 0)
    perm = ins["perm"] if wcols else np.arange(nnz)
    assert np.array_equal(np.sort(perm), np.arange(nnz))
    ranges = {w: (v0, v1) for w, v0, v1 in _check_blocks(ins, cap, T)}
    pcs = _pieces(rp, T)
    seen = {}
    nwin = len(ins["win_blk"]) - 1
    for w in range(nwin):
        if w not in ranges:
            continue
        v0, v1 = ranges[w]
        for v in range(v0, v1):
            src = perm[vp[v]:vp[v + 1]]
            if len(src):
                assert np.array_equal(src, np.arange(src[0], src[0] + len(src)))   # contiguous, in order
                if wcols:
                    assert np.all(col[src] // wcols == w)
            if wcols:
                code = int(vd[v])
                d, cont = code >> 1, code & 1
            else:
                d = int(vd[v]) if len(vd) else v
                cont = 0
            seg = seen.setdefault(d, [])
            assert cont == (1 if seg else 0), (d, w)
            seg.append(src)
    assert set(seen) == set(pcs)
    for d, (s, e) in pcs.items():
        got = np.concatenate(seen[d]) if seen[d] else np.zeros(0, np.int64)
        assert np.array_equal(got, np.arange(s, e)), d
    if wcols:
        assert nwin == (ncols + wcols - 1) // wcols
    else:
        assert nwin == 1


@pytest.mark.parametrize("name,rp,col,ncols", MATS[:1] + MATS[3:], ids=["gen", "handmade"])
def test_chained_emulation_bitwise(name, rp, col, ncols):
    """Emulate the chained launches (acc from the stored value, same op order) vs the unbroken row chain."""
    rng = np.random.default_rng(1)
    nnz, m, k, T = int(rp[-1]), len(rp) - 1, 3, 2048
    val = rng.uniform(-1, 1, nnz)
    B = rng.uniform(-1, 1, (ncols, k))
    want = np.zeros((m, k))
    for r in range(m):
        acc = np.zeros(k)
        for j in range(rp[r], rp[r + 1]):
            acc = acc + val[j] * B[col[j]]
        want[r] = acc
    ins = S.debug_inspect(rp, col, ncols, T, 2048, 97)
    vp, vd, perm, blk, wb = ins["vrow_ptr"], ins["vdest"], ins["perm"], ins["blk"], ins["win_blk"]
    Cm = np.full((m, k), np.nan)
    P = np.full((max(ins["nslots"], 1), k), np.nan)
    for w in range(len(wb) - 1):
        for b in range(wb[w], wb[w + 1]):
            for v in range(*blk[b]):
                code = int(vd[v])
                d = code >> 1
                dst = Cm[d] if d >= 0 else P[-d - 1]
                acc = dst.copy() if code & 1 else np.zeros(k)
                for q in range(vp[v], vp[v + 1]):
                    j = perm[q]
                    acc = acc + val[j] * B[col[j]]
                dst[:] = acc
    short = np.diff(rp) <= T
    assert np.array_equal(Cm[short].view(np.int64), want[short].view(np.int64))
    for row, s0, ns, _ in ins["long_rows"]:            # split rows: the pieces' partials sum to the row
        assert np.allclose(P[s0:s0 + ns].sum(0), want[row], rtol=1e-12, atol=1e-12)


def test_unsorted_rows_rejected_for_windows():
    rp = np.array([0, 3], np.int32)
    col = np.array([5, 1, 2], np.int32)
    with pytest.raises(S.SpmmHipError):
        S.debug_inspect(rp, col, 10, 64, 2048, 4)
    assert S.debug_inspect(rp, col, 10, 64, 2048, 0)["vrow_ptr"].tolist() == [0, 3]
