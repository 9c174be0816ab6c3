"""GPU parity of the matrix-core tile kernel (spmm_mfma_tile_kernel).

The f64 MFMA (v_mfma_f64_16x16x4_f64) accumulates its four products in k order, each one fused multiply-add, and a
zero of the panel adds fma(+0, b, acc) == acc: every row of a matrix-core tile is the reference's left-to-right chain
(compute_csr, spmm_kernel_csr.cpp:70-96).  So with matrix-core tiles forced (SPMM_HIP_MFMA=1) every row the engine
reports exact must be BIT-IDENTICAL to the oracle and to the row kernel (SPMM_HIP_TILES=-1).  Also: K panels
(K = 64, 96, 128), non-finite B values (the chunk is recomputed by the sparse chain: the reference's Inf/NaN and
nothing more), value updates, duplicate columns / fp32 / narrow panels (refused: another kernel runs), the default
policy on a dense band, and a captured hipGraph replay.
"""
import zlib

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


def handle(S, A, vals, k, monkeypatch, env):
    for kk in ("SPMM_HIP_TILES", "SPMM_HIP_MFMA", "SPMM_HIP_MFMA_REUSE", "SPMM_HIP_MFMA_RING"):
        monkeypatch.delenv(kk, raising=False)
    for kk, vv in env.items():
        monkeypatch.setenv(kk, vv)
    return S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)


def run(S, A, vals, x, k, monkeypatch, env):
    mf = handle(S, A, vals, k, monkeypatch, env)
    y = np.full(A.m * k, np.nan, vals.dtype)
    mf.spmm(np.ascontiguousarray(x, vals.dtype), y, k)
    ti, ex = mf.tile_info(), mf.exact_rows()
    mf.close()
    return y.reshape(A.m, k), ti, ex


MATS = ["6000 6000 100 33 normal random 0.05 0 0.95 0.95 14",          # similar rows
        "3000 3000 300 100 normal random 0.05 10 1.4 0.5 14",          # dense narrow band
        "20000 40000 10 3.3333 normal random 0.6 2000 0.5 0.95 3",     # a 20 K-nonzero split row + sparse tiles
        "4000 4000 40 13 normal random 0.6 0 0.05 0.05 14"]            # low reuse (density ~ 1/16)


@pytest.mark.parametrize("line", MATS, ids=["similar", "dense", "split", "lowreuse"])
@pytest.mark.parametrize("k", [32, 64, 96, 128])
@pytest.mark.parametrize("ring", ["12", "6"])     # B-operand slots per sub-panel: a whole chunk, or a 6-slot ring
def test_mfma_bitexact(env, monkeypatch, line, k, ring):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(7 + k, A.ncols * k) * 2.0 - 1.0          # mixed signs: rounding in every chain
    y1, t1, ex1 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1", "SPMM_HIP_MFMA_RING": ring})
    assert t1["mode"] == "mfma" and t1["tiles"] > 0
    y0, t0, ex0 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_TILES": "-1"})
    assert t0["tiles"] == 0
    both = ex0 & ex1
    assert both.sum() >= t1["rows"] * 0.99
    assert np.array_equal(bits(y1[both]), bits(y0[both]))
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(bits(y1[ex1]), bits(seq[ex1]))
    if (~ex1).any():
        g, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
        assert O.normwise_ok(y1[~ex1], g[~ex1], absdot[~ex1], 1e-10).all()


def test_mfma_nonfinite_b(env, monkeypatch):
    """Inf / NaN in B: a panel zero times them must not leak into rows that do not use those B rows."""
    torch, S, O = env
    A = S.generate(S.gen_params("6000 6000 100 33 normal random 0.05 0 0.95 0.95 14"))
    k = 32
    x = O.drand48(3, A.ncols * k).reshape(k, A.ncols)      # column-major: x[n][col]
    cols = np.unique(A.col_idx)
    rng = np.random.default_rng(4)
    x[rng.integers(0, k, 6), rng.choice(cols, 6)] = np.inf
    x[rng.integers(0, k, 6), rng.choice(cols, 6)] = -np.inf
    x[rng.integers(0, k, 6), rng.choice(cols, 6)] = np.nan
    x = x.reshape(-1)
    y1, t1, ex1 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t1["mode"] == "mfma"
    seq = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(np.isnan(y1[ex1]), np.isnan(seq[ex1]))
    fin = ~np.isnan(seq[ex1])
    assert np.array_equal(bits(y1[ex1][fin]), bits(seq[ex1][fin]))
    assert np.isfinite(seq).sum() > 0.9 * seq.size           # most rows never touch the planted values


def test_mfma_refused(env, monkeypatch):
    """K not a multiple of 32 and repeated columns never take matrix-core tiles (another kernel runs, still exact)."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[1]))
    for vals, k in ((A.values.astype(np.float32), 48), (A.values, 8)):
        mf = handle(S, A, vals, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
        assert mf.tile_info()["mode"] != "mfma"
        mf.close()
    # a repeated column in one row (duplicate .mtx entries are kept, not summed)
    rp, ci = A.row_ptr.copy(), A.col_idx.copy()
    ci[rp[5] + 1] = ci[rp[5]]
    B2 = S.CSR(rp, ci, A.values.copy(), A.m, A.ncols)
    x = O.drand48(5, A.ncols * 32)
    y, t, ex = run(S, B2, B2.values, x, 32, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t["mode"] != "mfma"
    seq = O.spmm(B2.row_ptr, B2.col_idx, B2.values, B2.ncols, x, 32)
    assert np.array_equal(bits(y[ex]), bits(seq[ex]))


def test_mfma_update_values(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[0]))
    k = 64
    x = O.drand48(6, A.ncols * k)
    mf = handle(S, A, A.values, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert mf.tile_info()["mode"] == "mfma"
    v2 = np.random.default_rng(9).uniform(-1, 1, A.nnz)
    mf.update_values(v2)
    y = np.zeros(A.m * k)
    mf.spmm(x, y, k)
    ex = mf.exact_rows()
    mf.close()
    want = O.spmm(A.row_ptr, A.col_idx, v2, A.ncols, x, k)
    assert np.array_equal(bits(y.reshape(A.m, k)[ex]), bits(want[ex]))


def test_mfma_policy_dense_band(env, monkeypatch):
    """Default policy: the plan takes matrix-core tiles exactly when the gate (spmm_hip_debug_plan, host only) says
    so -- on dense bands at K = 32 and 128 -- and the gate forced open (SPMM_HIP_MFMA=2) always takes them there; a
    low-reuse matrix does not."""
    torch, S, O = env
    for line in ("22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14",
                 "111476 111476 100 33.3333 normal random 0.3 0 0.05 0.95 14"):
        A = S.generate(S.gen_params(line))
        for k in (32, 128):
            d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, gate_only=True)
            mf = handle(S, A, A.values, k, monkeypatch, {})
            assert mf.tile_info()["mode"] == ("mfma" if d["gate"] else mf.tile_info()["mode"]), (line, k)
            assert (mf.tile_info()["mode"] == "mfma") == bool(d["gate"]), (line, k)
            mf.close()
            mf = handle(S, A, A.values, k, monkeypatch, {"SPMM_HIP_MFMA": "2"})
            assert mf.tile_info()["mode"] == "mfma", (line, k)
            mf.close()
    L = S.generate(S.gen_params("200000 200000 10 3.3333 normal random 0.6 0 0.05 0.05 14"))
    mf = handle(S, L, L.values, 32, monkeypatch, {})
    assert mf.tile_info()["mode"] != "mfma"
    mf.close()


def test_mfma_graph_replay(env, monkeypatch):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[1]))
    k = 32
    mf = handle(S, A, A.values, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert mf.tile_info()["mode"] == "mfma"
    dev = torch.device("cuda", 0)
    B = torch.rand((A.ncols, k), dtype=torch.float64, device=dev)
    C1 = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    C2 = torch.empty_like(C1)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C1.data_ptr(), k, s.cuda_stream)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C2.data_ptr(), k, s.cuda_stream)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(C1.view(torch.int64), C2.view(torch.int64))
    mf.close()


def test_mfma_range_check_per_launch(env, monkeypatch):
    """B's exact-range check is per launch: launches alternating in-range and out-of-range B (NaN, a
    subnormal) on one handle -- each exact row bit-identical to the oracle (NaN where the oracle has NaN), so the
    fix-up neither sticks after a bad B nor is skipped after a good one; and a captured graph replayed after its B
    turned in-range and out-of-range again stays exact (a baked-in launch number can only keep the fix-up on)."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[0]))
    k = 32
    mf = handle(S, A, A.values, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert mf.tile_info()["mode"] == "mfma"
    ex = mf.exact_rows()
    dev = torch.device("cuda", 0)
    base = O.drand48(11, A.ncols * k).reshape(A.ncols, k) * 2.0 - 1.0
    cols = np.unique(A.col_idx)
    bad_nan, bad_sub = base.copy(), base.copy()
    bad_nan[cols[len(cols) // 2], 3] = np.nan
    bad_sub[cols[len(cols) // 3], 5] = 2.0 ** -1060
    want = {}
    for name, xb in (("ok", base), ("nan", bad_nan), ("sub", bad_sub)):
        want[name] = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, np.ascontiguousarray(xb.T).reshape(-1), k)
    B = torch.empty((A.ncols, k), dtype=torch.float64, device=dev)
    C = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)

    def check(name):
        got = C.cpu().numpy()[ex]
        w = want[name][ex]
        assert np.array_equal(np.isnan(got), np.isnan(w)), name
        fin = ~np.isnan(w)
        assert np.array_equal(bits(got[fin]), bits(w[fin])), name

    src = {"ok": base, "nan": bad_nan, "sub": bad_sub}
    for name in ("ok", "nan", "ok", "sub", "ok", "ok", "nan", "ok"):
        B.copy_(torch.from_numpy(src[name]))
        C.fill_(7.0)
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, st.cuda_stream)
        torch.cuda.synchronize()
        check(name)
    s = torch.cuda.Stream(dev)
    B.copy_(torch.from_numpy(bad_nan))
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, s.cuda_stream)
    for name in ("nan", "ok", "sub", "ok"):
        B.copy_(torch.from_numpy(src[name]))
        C.fill_(7.0)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        check(name)
    mf.close()


# ---------------------------------------------------------------------------------------------------------------
# IEEE edge cases (spmm_mfma.hpp header: the exact-chain range check).  The reference sums each row as one chain of
# fused multiply-adds from +0 in IEEE double on x86 (spmm_kernel_csr.cpp:87-91): subnormal operands and products,
# underflow to -0, -0 inputs and overflow all follow IEEE there.  A matrix-core tile adds fma(0, b, acc) steps for
# its empty panel cells, which could turn a -0 chain into +0 and which would expose a flush-to-zero of subnormals;
# the kernel therefore recomputes any tile whose operands leave 2^-458 <= |x| <= 2^500 by the sparse IEEE chain.
# Rows the engine reports exact must be bit-identical to the oracle for every kind of value below, with matrix-core
# tiles forced, with the LDS tile kernel forced (padding entries -0 on the zero B row) and with the row kernel.

def edge_values(kind, n, rng):
    """(A values, B values) of one edge-case family; n = (nnz, B entries)."""
    na, nb = n
    sa = rng.choice([-1.0, 1.0], na)
    sb = rng.choice([-1.0, 1.0], nb)
    ua, ub = rng.uniform(0.5, 1.5, na), rng.uniform(0.5, 1.5, nb)
    if kind == "subnormal_a":        # A subnormal (2^-1070 .. 2^-1030), B ~ 1 .. 2^60: products subnormal or normal
        return sa * ua * 2.0 ** rng.integers(-1070, -1030, na), sb * ub * 2.0 ** rng.integers(0, 60, nb)
    if kind == "subnormal_b":
        return sa * ua * 2.0 ** rng.integers(0, 60, na), sb * ub * 2.0 ** rng.integers(-1070, -1030, nb)
    if kind == "underflow":          # products ~ 2^-1040 .. 2^-1090: subnormal partial sums, underflow to +-0
        return sa * ua * 2.0 ** rng.integers(-545, -520, na), sb * ub * 2.0 ** rng.integers(-545, -520, nb)
    if kind == "negzero":            # -0 / +0 entries and tiny negative products: -0 chains
        a = sa * ua * 2.0 ** -540
        b = sb * ub * 2.0 ** -540
        a[rng.random(na) < 0.3] = -0.0
        b[rng.random(nb) < 0.3] = -0.0
        a[rng.random(na) < 0.1] = 0.0
        return a, b
    if kind == "near_range":         # just inside / outside the exact range bounds 2^-458, 2^500
        return sa * 2.0 ** rng.choice([-459, -458, -457, 0, 499, 500], na), sb * 2.0 ** rng.choice([-459, -458, 0, 1], nb)
    if kind == "overflow":           # products beyond DBL_MAX: +-Inf, Inf - Inf = NaN
        return sa * ua * 2.0 ** rng.integers(480, 530, na), sb * ub * 2.0 ** rng.integers(480, 530, nb)
    if kind == "mixed":              # per entry one of normal / tiny / zero / -0 / subnormal
        a, b = sa * ua, sb * ub
        for v in (a, b):
            c = rng.integers(0, 5, len(v))
            v[c == 1] *= 2.0 ** -1060
            v[c == 2] *= 2.0 ** -530
            v[c == 3] = 0.0
            v[c == 4] = -0.0
        return a, b
    raise ValueError(kind)


EDGE_KINDS = ["subnormal_a", "subnormal_b", "underflow", "negzero", "near_range", "overflow", "mixed"]
EDGE_PLANS = {"mfma": {"SPMM_HIP_MFMA": "1"}, "lds": {"SPMM_HIP_MFMA": "-1", "SPMM_HIP_TILES": "1"},
              "rows": {"SPMM_HIP_TILES": "-1"}}


def same_bits_or_nan(got, want):
    """Bit-identical, except that a NaN only has to be a NaN (x86 and the GPU make NaNs with different sign bits)."""
    gn, wn = np.isnan(got), np.isnan(want)
    return np.array_equal(gn, wn) and np.array_equal(bits(got[~gn]), bits(want[~wn]))


@pytest.mark.parametrize("kind", EDGE_KINDS)
@pytest.mark.parametrize("plan", list(EDGE_PLANS))
@pytest.mark.parametrize("k", [32, 64])
def test_edge_values_exact(env, monkeypatch, kind, plan, k):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[0]))
    rng = np.random.default_rng(zlib.crc32(f"{kind}/{k}".encode()))
    vals, x = edge_values(kind, (A.nnz, A.ncols * k), rng)
    y, t, ex = run(S, A, vals, x, k, monkeypatch, EDGE_PLANS[plan])
    if plan == "mfma":
        assert t["mode"] == "mfma" and t["rows"] > 0.9 * A.m
    elif plan == "lds":
        assert t["mode"] == "lds" and t["rows"] > 0.5 * A.m
    else:
        assert t["tiles"] == 0
    want = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
    assert ex.sum() > 0.99 * A.m
    assert same_bits_or_nan(y[ex], want[ex]), f"{kind}: {plan} rows differ from the reference chain"
    if kind in ("underflow", "negzero", "mixed"):          # the family really exercised signed zeros / subnormals
        z = want[ex]
        assert (np.signbit(z) & (z == 0)).any() or (np.abs(z[z != 0]) < 2.0 ** -1022).any()


def test_mfma_edge_tile_only_falls_back(env, monkeypatch):
    """One tiny B value makes only the tiles that read it take the sparse chain: all rows still exact and equal."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[1]))
    k = 32
    x = O.drand48(11, A.ncols * k) * 2.0 - 1.0
    x[5] = 2.0 ** -1070                      # one subnormal in B column 5 (column-major: x[n][col], n = 0)
    x[7 * A.ncols + 40] = -0.0
    y, t, ex = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t["mode"] == "mfma"
    want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(bits(y[ex]), bits(want[ex]))


def test_mfma_leftover_rows_keep_exactness(env, monkeypatch):
    """ When tiles hold nearly all nonzeros only the rows longer than T are cut into 64-nonzero pieces: the
    exact-row mask equals the plan without matrix-core tiles, and those rows equal the oracle."""
    torch, S, O = env
    A = S.generate(S.gen_params("6000 6000 100 33 normal random 0.05 60 0.95 0.95 14"))
    k = 32
    x = O.drand48(2, A.ncols * k)
    y1, t1, ex1 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    y0, t0, ex0 = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_TILES": "-1"})
    assert t1["mode"] == "mfma" and t1["nnz"] > 0.875 * A.nnz
    assert (~ex0).sum() >= 1                                 # the skewed row is split in both plans
    assert np.array_equal(ex1, ex0)
    want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert np.array_equal(bits(y1[ex1]), bits(want[ex1]))
    g, absdot = O.gold(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    assert O.normwise_ok(y1[~ex1], g[~ex1], absdot[~ex1], 1e-10).all()


@pytest.mark.parametrize("np_env", ["1", "2"])
def test_mfma_wave_panels_bitexact(env, monkeypatch, np_env):
    """64-column waves (NP = 2) and 32-column waves give the same bits at K = 64, 96, 128, 160."""
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[0]))
    monkeypatch.setenv("SPMM_HIP_MFMA_NP", np_env)
    for k in (64, 96, 160):
        x = O.drand48(k, A.ncols * k) * 2.0 - 1.0
        y, t, ex = run(S, A, A.values, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
        assert t["mode"] == "mfma"
        want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
        assert np.array_equal(bits(y[ex]), bits(want[ex])), k


def test_multi_handle_tile_mode(env, monkeypatch):
    """ A multi-GPU handle reports the tile kernel its shards run."""
    torch, S, O = env
    monkeypatch.setenv("SPMM_HIP_MFMA", "1")
    A = S.generate(S.gen_params(MATS[0]))
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, 32, 0, devices=[0, 0])
    ti = mf.tile_info()
    assert ti["tiles"] > 0 and ti["mode"] == "mfma"
    mf.close()


def test_debug_plan_matches_handle(env, monkeypatch):
    """spmm_hip_debug_plan (host only) reports what the handle planned."""
    torch, S, O = env
    for kk in ("SPMM_HIP_TILES", "SPMM_HIP_MFMA", "SPMM_HIP_MFMA_REUSE", "SPMM_HIP_MFMA_RING"):
        monkeypatch.delenv(kk, raising=False)
    for line in ("22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14", MATS[2]):
        A = S.generate(S.gen_params(line))
        for k in (32, 128):
            d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k)
            mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
            ti, inf = mf.tile_info(), mf.info()
            assert d["mode"] == ti["mode"] and d["ntile"] == ti["tiles"] and d["tile_nnz"] == ti["nnz"]
            assert d["seq_max"] == inf[8] and d["blocks"] == inf[5] and d["exact_rows"] == inf[17]
            mf.close()


# ---------------------------------------------------------------------------------------------------------------
# fp32 matrix-core tiles: v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain (tools/mfma_chain_probe.py,
# profiles/r04/chain_probe.jsonl), so fp32 tile rows equal the reference FLOAT build's chain (the oracle's fp32 path is
# pinned to it, tests/test_oracle_golden.py) bit for bit.

@pytest.mark.parametrize("line", MATS, ids=["similar", "dense", "split", "lowreuse"])
@pytest.mark.parametrize("k", [32, 64, 128])
@pytest.mark.parametrize("ring", ["12", "6"])
def test_mfma_f32_bitexact(env, monkeypatch, line, k, ring):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    vals = (A.values * np.where(np.arange(A.nnz) % 3 == 0, -1.0, 1.0)).astype(np.float32)
    x = (O.drand48(17 + k, A.ncols * k) * 2.0 - 1.0).astype(np.float32)
    y1, t1, ex1 = run(S, A, vals, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1", "SPMM_HIP_MFMA_RING": ring})
    assert t1["mode"] == "mfma" and t1["tiles"] > 0
    assert ex1.sum() >= t1["rows"] * 0.99                # tile rows are exact rows
    y0, t0, ex0 = run(S, A, vals, x, k, monkeypatch, {"SPMM_HIP_TILES": "-1"})
    both = ex0 & ex1          # (the row kernel may give a small long-row fp32 matrix vector lanes: no exact rows)
    assert np.array_equal(bits(y1[both]), bits(y0[both]))
    seq = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
    assert np.array_equal(bits(y1[ex1]), bits(seq[ex1]))


def edge_values_f32(kind, n, rng):
    na, nb = n
    sa, sb = rng.choice([-1.0, 1.0], na), rng.choice([-1.0, 1.0], nb)
    ua, ub = rng.uniform(0.5, 1.5, na), rng.uniform(0.5, 1.5, nb)
    if kind == "subnormal":          # f32 subnormals (2^-149 .. 2^-127) against values up to 2^30
        a, b = sa * ua * 2.0 ** rng.integers(-145, -128, na), sb * ub * 2.0 ** rng.integers(0, 30, nb)
    elif kind == "underflow":        # products 2^-150 .. 2^-110: subnormal sums, underflow to +-0
        a, b = sa * ua * 2.0 ** rng.integers(-75, -55, na), sb * ub * 2.0 ** rng.integers(-75, -55, nb)
    elif kind == "near_range":       # around the fp32 bound 2^-40
        a, b = sa * 2.0 ** rng.choice([-41, -40, -39, 0, 60], na), sb * 2.0 ** rng.choice([-41, -40, 0, 1], nb)
    elif kind == "overflow":
        a, b = sa * ua * 2.0 ** rng.integers(60, 70, na), sb * ub * 2.0 ** rng.integers(60, 70, nb)
    else:
        raise ValueError(kind)
    return a.astype(np.float32), b.astype(np.float32)


@pytest.mark.parametrize("kind", ["subnormal", "underflow", "near_range", "overflow"])
def test_mfma_f32_edge_values(env, monkeypatch, kind):
    torch, S, O = env
    A = S.generate(S.gen_params(MATS[0]))
    k = 32
    rng = np.random.default_rng(zlib.crc32(f"f32/{kind}".encode()))
    vals, x = edge_values_f32(kind, (A.nnz, A.ncols * k), rng)
    y, t, ex = run(S, A, vals, x, k, monkeypatch, {"SPMM_HIP_MFMA": "1"})
    assert t["mode"] == "mfma"
    want = O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k)
    assert same_bits_or_nan(y[ex], want[ex]), kind
