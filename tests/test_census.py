"""CPU tests of the host-only planner (spmm_hip_debug_plan) and the dataset census built on it (tools/plan_census.py).

The census evaluates the matrix-core gate of every medium-dataset line from the gate's sampled
16-row tiles only: the matrix is generated for those rows (spmm_host_generate_masked) and the gate must decide
exactly as it does on the full matrix.  A line the gate keeps off must plan exactly as the engine without
matrix-core tiles (SPMM_HIP_MFMA=-1: the config-3 sweep build's plan) -- same plan fingerprint.
"""
import numpy as np
import pytest

LINES = ["22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14",      # dense band: tiles
         "39120 39120 500 166.6667 normal random 0.05 0 0.05 0.5 14",
         "111476 111476 100 33.3333 normal random 0.3 0 0.5 0.95 14",
         "250000 250000 20 6.6667 normal random 0.3 100 0.95 0.5 14",       # config-2-like: no tiles
         "4000 4000 40 13 normal random 0.6 0 0.05 0.05 14"]


@pytest.fixture(scope="module")
def S():
    import spmm_amd
    return spmm_amd


@pytest.mark.parametrize("line", LINES)
def test_masked_generation_equals_full(S, line):
    p = S.gen_params(line)
    A = S.generate(p)
    mask = S.gate_sample_rows(A.m)
    M = S.generate_masked(p, mask)
    assert np.array_equal(M.row_ptr, A.row_ptr)
    sel = np.repeat(mask.astype(bool), np.diff(A.row_ptr))
    assert np.array_equal(M.col_idx[sel], A.col_idx[sel]) and np.array_equal(M.values[sel], A.values[sel])


@pytest.mark.parametrize("line", LINES)
@pytest.mark.parametrize("k", [32, 128])
def test_gate_from_sample_equals_full(S, line, k):
    """The gate reads its sampled rows only: masked columns and full columns give the same decision and statistics,
    and the full plan takes matrix-core tiles exactly when the gate says so."""
    p = S.gen_params(line)
    A = S.generate(p)
    M = S.generate_masked(p, S.gate_sample_rows(A.m))
    g_full = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, gate_only=True)
    g_mask = S.debug_plan(M.row_ptr, M.col_idx, M.ncols, k, gate_only=True)
    for f in ("mode", "gate", "r16", "take", "est_tile_nnz", "est_chunks", "t_on_us", "t_off_us", "seq_max"):
        assert g_full[f] == g_mask[f], f
    full = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k)
    assert (full["mode"] == "mfma") == (g_full["mode"] == "mfma")
    off = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, mfma=-1)
    assert off["mode"] != "mfma"
    # unchanged vs the plan without matrix-core tiles exactly when the gate is off
    assert (full["fingerprint"] == off["fingerprint"]) == (full["mode"] != "mfma")


def test_debug_plan_estimates(S):
    """The gate's sample estimates the built tiles: nonzeros in tiles within 5 %, chunks within 10 %."""
    A = S.generate(S.gen_params(LINES[0]))
    d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, 32, mfma=2)          # the gate forced open
    assert d["mode"] == "mfma"
    assert abs(d["est_tile_nnz"] / d["tile_nnz"] - 1) < 0.05
    assert abs(d["est_chunks"] / d["tile_chunks"] - 1) < 0.10


def test_debug_plan_forced_modes(S):
    A = S.generate(S.gen_params(LINES[4]))
    assert S.debug_plan(A.row_ptr, A.col_idx, A.ncols, 32, mfma=1)["mode"] == "mfma"
    assert S.debug_plan(A.row_ptr, A.col_idx, A.ncols, 32, mfma=-1)["mode"] != "mfma"
    f32 = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, 32, dtype=S.F32, mfma=1)
    assert f32["mode"] == "mfma"                         # fp32 matrix-core tiles (v_mfma_f32_16x16x4_f32)
    assert S.debug_plan(A.row_ptr, A.col_idx, A.ncols, 8, mfma=1)["mode"] != "mfma"   # K not a multiple of 32


def test_debug_plan_rejects_bad_input(S):
    rp = np.array([0, 2, 1], np.int32)
    with pytest.raises(S.SpmmHipError):
        S.debug_plan(rp, np.zeros(2, np.int32), 4, 32)
    with pytest.raises(S.SpmmHipError):
        S.debug_plan(np.array([0, 1], np.int32), np.array([7], np.int32), 4, 32)


@pytest.mark.parametrize("line", LINES[:3])
def test_debug_gate_reproduces_plan_verdict(S, line):
    """spmm_hip_debug_gate on the sample debug_plan reports gives debug_plan's own verdict and model times."""
    A = S.generate(S.gen_params(line))
    for dt in (S.F64, S.F32):
        for k in (32, 64, 128):
            d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, dtype=dt, gate_only=True)
            g = S.debug_gate(A.m, A.nnz, k, d, dtype=dt)
            assert g["gate"] == d["gate"] and g["t_on_us"] == d["t_on_us"] and g["t_off_us"] == d["t_off_us"]


def test_plan_without_tiles_is_config3_plan():
    """The plan without matrix-core tiles (SPMM_HIP_MFMA=-1) reproduces the plans the config-3 sweep build recorded
    (engine b4d29bad, profiles/r03_sweep_medium.jsonl.gz) -- on a sparse stride sample of small lines, all K."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    if not (root / "profiles" / "r03_sweep_medium.jsonl.gz").exists():
        pytest.skip("config-3 sweep records not present")
    sys.path.insert(0, str(root / "tools"))
    import plan_vs_r03
    res = plan_vs_r03.compare(stride=997, max_nnz=3e6, workers=1)
    assert len(res) >= 20
    assert [r for r in res if r[2]] == []


def test_gate_only_checks_sampled_columns(S):
    """Gate-only mode reads the sampled rows' columns only -- and range-checks them (they index host arrays of ncols
    entries); a bad column outside the sample is never read."""
    p = S.gen_params(LINES[3])
    A = S.generate(p)
    mask = S.gate_sample_rows(A.m).astype(bool)
    sel = np.repeat(mask, np.diff(A.row_ptr))
    inside, outside = np.flatnonzero(sel), np.flatnonzero(~sel)
    assert len(inside) and len(outside)
    for j, bad in ((inside[len(inside) // 2], True), (outside[len(outside) // 2], False)):
        for v in (-1, A.ncols):
            col = A.col_idx.copy()
            col[j] = v
            if bad:
                with pytest.raises(RuntimeError, match="out of range"):
                    S.debug_plan(A.row_ptr, col, A.ncols, 32, gate_only=True)
            else:
                S.debug_plan(A.row_ptr, col, A.ncols, 32, gate_only=True)
