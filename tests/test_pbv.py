"""The perfect-balance K = 1 format (include/spmm_pbv.h) on the host: its plan (block starts by the merge-path
search, the exact-row mask) against a restatement written from the definitions, and its factory failing loudly
without a GPU.  The device kernel is checked against the oracle in tests/test_gpu_pbv.py.

Definitions (spmv_pbv.hip): items = m row ends + nnz nonzeros in CSR order (row end i after the nonzeros of row i);
block b = items [b*256E, (b+1)*256E); lane = E consecutive items.  The block start is the split {row ends consumed,
nonzeros consumed} after d = b*256E items.  A row is exact when its first nonzero item and its row-end item are in
one lane (its whole chain runs in that lane from 0).
"""
import numpy as np
import pytest

import spmm_amd as S
import spmm_amd.pbv as P


def item_stream(rp):
    """[(kind, row)] in merge order: ('nz', row) per nonzero, ('end', row) per row end."""
    out = []
    for r in range(len(rp) - 1):
        out += [("nz", r)] * int(rp[r + 1] - rp[r]) + [("end", r)]
    return out


def restated_plan(rp, e):
    m, nnz = len(rp) - 1, int(rp[-1])
    items = item_stream(rp)
    per = 256 * e
    nblk = -(-(m + nnz) // per) if m else 0
    blk = []
    for b in range(nblk + 1):
        d = min(b * per, m + nnz)
        ends = sum(1 for kind, _ in items[:d] if kind == "end")
        blk.append((ends, d - ends))
    exact = []
    for r in range(m):
        pos = [i for i, (kind, row) in enumerate(items) if row == r]
        exact.append(pos[0] // e == pos[-1] // e)
    return np.array(blk, np.int32).reshape(-1, 2), np.array(exact, bool)


def random_rp(rng, m, kind):
    if kind == "uniform":
        deg = rng.integers(0, 12, m)
    elif kind == "empty_runs":                 # long runs of empty rows between a few dense ones
        deg = np.where(rng.random(m) < 0.05, rng.integers(50, 400, m), 0)
    elif kind == "giant":                      # one row spanning many blocks
        deg = rng.integers(0, 4, m)
        deg[m // 3] = 9000
    else:
        deg = rng.zipf(1.6, m).clip(0, 3000)
    return np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)


@pytest.mark.parametrize("e", [4, 8, 16])
@pytest.mark.parametrize("kind", ["uniform", "empty_runs", "giant", "zipf"])
def test_plan_matches_restatement(e, kind):
    rng = np.random.default_rng(hash((e, kind)) % 2**32)
    rp = random_rp(rng, 1500, kind)
    blk, ex = P.plan_host(rp, len(rp) - 1, int(rp[-1]), e)
    want_blk, want_ex = restated_plan(rp, e)
    assert np.array_equal(blk, want_blk)
    assert np.array_equal(ex, want_ex)
    # every block holds exactly 256 E items except the last
    d = blk.sum(axis=1)
    assert (np.diff(d)[:-1] == 256 * e).all() and 0 < d[-1] - d[-2] <= 256 * e


def test_plan_edge_cases():
    blk, ex = P.plan_host(np.zeros(1, np.int32), 0, 0, 8)           # m = 0: no blocks
    assert blk.shape == (1, 2) and ex.size == 0
    rp = np.zeros(5001, np.int32)                                     # nnz = 0: row ends only, all exact
    blk, ex = P.plan_host(rp, 5000, 0, 8)
    assert blk.tolist()[-1] == [5000, 0] and ex.all() and len(blk) == 4
    rp = np.array([0, 7], np.int32)                                   # one row of 7 + its end = 8 items: one lane
    assert P.plan_host(rp, 1, 7, 8)[1].tolist() == [True]
    rp = np.array([0, 8], np.int32)                                   # 9 items: cut
    assert P.plan_host(rp, 1, 8, 8)[1].tolist() == [False]
    with pytest.raises(S.SpmmHipError):
        P.plan_host(rp, 1, 8, 3)                                      # E outside [4, 16]


def test_factory_fails_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible: tests/test_gpu_pbv.py covers the device path")
    except ImportError:
        pass
    rp = np.array([0, 1, 2], np.int32)
    with pytest.raises(S.SpmmHipError) as e:
        P.PBVFormat(rp, np.array([0, 1], np.int32), np.ones(2), 2, 2, 2)
    assert e.value.status == -4                                       # no HIP device: no CPU fallback
    with pytest.raises(S.SpmmHipError) as e:                          # malformed CSR is refused before the device
        P.PBVFormat(np.array([0, 2, 1], np.int32), np.array([0, 1], np.int32), np.ones(2), 2, 2, 2)
    assert e.value.status == -6
