"""bench.py helpers on CPU: the gather-ceiling model, the per-matrix PMC records' engine keying, and
the dataset summary's aggregates."""
import json
import math

import pytest

import bench


def test_gather_rate_interpolates_the_probe():
    for b, r in bench.GATHER_PROBE:
        assert math.isclose(bench.gather_rate_tbs(b), r, rel_tol=1e-9)
    assert bench.gather_rate_tbs(1 << 10) == bench.GATHER_PROBE[0][1]          # below the probe: L2-resident rate
    assert bench.gather_rate_tbs(1 << 40) == bench.GATHER_PROBE[-1][1]         # beyond: the HBM rate
    mid = bench.gather_rate_tbs(32 << 20)
    assert bench.GATHER_PROBE[2][1] < mid < bench.GATHER_PROBE[1][1]


def test_achievable_takes_the_larger_bound():
    # config 2 of round 3: 3.13 GB past L2, 34.2 M L2 requests, B of 256 MB, 0.416 ms measured
    a = bench.achievable(0.41565, 3.131956852e9, 34.18e6, 1e6 * 32 * 8)
    assert a["bound"] == "past-L2 gather"
    assert a["t_ms"] == pytest.approx(3.131956852e9 / (bench.gather_rate_tbs(256e6) * 1e12) * 1e3, rel=1e-4)
    assert a["frac_of_achievable"] == pytest.approx(a["t_ms"] / 0.41565, rel=1e-3)
    b = bench.achievable(1.0, 1e6, 1e9, 1e6)                   # few past-L2 bytes, many L2 requests
    assert b["bound"] == "L2 requests" and b["t_l2_ms"] > b["t_past_l2_ms"]
    assert bench.achievable(1.0, None, None, 1e6) is None


def test_achievable_never_below_the_hbm_roofline_time():
    """K = 1, 72652 x 500 (round-5 PMC): 0.437 GB of compulsory bytes, past-L2 traffic 1.04x of them, B 0.6 MB.  The
    gather terms price that stream at the L2-resident rate (a 0.024-ms "ceiling"); the HBM term keeps the ceiling at
    or above the roofline time of the compulsory bytes."""
    alg = 437.0e6
    a = bench.achievable(0.1042, 1.04 * alg, 5.29e6, 72652 * 8, alg)
    assert a["bound"] == "HBM compulsory"
    assert a["t_ms"] == pytest.approx(alg / 8e12 * 1e3, rel=1e-3) and a["t_hbm_ms"] == a["t_ms"]
    assert a["t_ms"] > max(a["t_past_l2_ms"], a["t_l2_ms"])
    b = bench.achievable(0.41565, 3.131956852e9, 34.18e6, 1e6 * 32 * 8, 755999464.0)   # config 2: gather-bound
    assert b["bound"] == "past-L2 gather" and b["t_hbm_ms"] < b["t_ms"]


def test_pmc_dataset_records_are_keyed_by_engine_build(tmp_path):
    sha = bench.engine_sha256()
    recs = [{"gen": "a", "k": 32, "dtype": "f64", "engine_sha256": sha, "traffic_bytes": 1.0},
            {"gen": "b", "k": 32, "dtype": "f64", "engine_sha256": "0" * 64, "traffic_bytes": 2.0},
            {"gen": "c", "k": 8, "dtype": "f64", "engine_sha256": sha, "traffic_bytes": 3.0}]
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"engine_sha256": sha, "records": recs}))
    got = bench.load_pmc_dataset(str(p), 32, "f64")
    assert set(got) == {"a"}
    assert bench.load_pmc_dataset(str(tmp_path / "missing.json"), 32, "f64") == {}


def test_summarize_aggregates():
    recs = [{"flops": 2e9, "ms": 1.0, "bytes_alg": 1e9, "frac": 0.125, "gflops": 2000.0, "traffic": 3e9,
             "frac_of_achievable": 0.5, "cpu_ms": 100.0},
            {"flops": 6e9, "ms": 1.0, "bytes_alg": 3e9, "frac": 0.375, "gflops": 6000.0}]
    s = bench.summarize({"recs": recs, "bad": 0, "wall_s": 1.0, "threads": 16, "model": "x"}, 32)
    assert s["value"] == pytest.approx(4000.0)                 # sum flops / sum time
    assert s["roofline"]["achieved"] == pytest.approx(2000.0)  # sum bytes / sum time
    assert s["roofline"]["traffic"] == 3e9 and s["roofline"]["achievable"]["matrices"] == 1
    assert s["cpu_baseline"]["value"] == pytest.approx(20.0) and "1 of the 2" in s["cpu_baseline"]["sample"]


def test_oracle_compare_bitexact_rows_and_tolerance():
    """The dataset leg's check of the GPU's C against the CPU baseline's oracle output: exact rows must match bit
    for bit, the others within the normwise contract."""
    import numpy as np
    import spmm_amd as S
    from oracle import oracle as O
    A = S.generate(S.gen_params("300 300 20 5 normal random 0.3 0 0.5 0.5 14"))
    k = 4
    x = O.drand48(3, A.ncols * k) - 0.5
    want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
    ex = np.ones(A.m, np.uint8)
    r = bench.oracle_compare(A, x, k, want.copy(), want, ex, np.float64)
    assert r["ok"] and r["rows_exact"] == A.m and r["exact_mismatch"] == 0
    got = want.copy()
    got[3, 1] = np.nextafter(got[3, 1], np.inf)                 # one ulp off on an exact row: a failure
    r = bench.oracle_compare(A, x, k, got, want, ex, np.float64)
    assert not r["ok"] and r["exact_mismatch"] == 1
    ex[3] = 0                                                    # the same row reported inexact: within tolerance
    r = bench.oracle_compare(A, x, k, got, want, ex, np.float64)
    assert r["ok"] and r["rows_inexact"] == 1
    got[3, 1] += 1.0                                             # far off: outside it
    r = bench.oracle_compare(A, x, k, got, want, ex, np.float64)
    assert not r["ok"] and r["inexact_outside_tol"] == 1
