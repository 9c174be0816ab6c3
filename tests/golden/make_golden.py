"""tests/golden/make_golden.py -- regenerate the golden fixtures FROM THE REFERENCE ITSELF.

Run in the container that has /root/reference, after `make -C oracle` built oracle/_ref/:
    python tests/golden/make_golden.py

What it writes (data only -- inputs and the reference's outputs; no reference source):
  mtx/*.mtx                 hand-written Matrix Market inputs covering the reader's cases
                            (general/symmetric/skew/Hermitian; real/integer/complex/pattern; empty rows; duplicates;
                            one long row; unsorted entries)
  smtx_csr.npz              per DLMC .smtx (tests/golden/smtx/): the offsets / columns smtx_read returns
  mtx_csr.npz               per .mtx: the CSR that mtx_read + coo_to_csr produce (spmv_bench.cpp:724-826), and
                            C = A*B from the reference plugin for K in {1,4,32} with B = 1 and B = drand48(42)
  mtx_csr_f32.npz           the same from the reference's FLOAT build (ValueType=float): values as it reads them,
                            C for K in {1,4,32} with x = (float) drand48(42)
  spmm_cases.npz            seeded random CSRs (empty rows, a long row, a zero-nnz matrix) and the reference
                            plugin's C for fp64 and fp32 at K in {1,8,32,128}
  partition.npz             loop_partitioner_balance_prefix_sums boundaries for several row_ptr / worker counts
  metrics.npz               the 8 CheckAccuracy metrics (array_metrics) on (gold, test) pairs
  features.npz              CSR patterns (the .mtx fixtures, hand-made edge cases, generator outputs) and what the
                            reference's feature extractor (csr_matrix_features_validation, csr_util_gen.c:889-990)
                            reports for them: avg, std, bw, skew, neighbours, cross-row similarity (the twin line)

Every value in these files was computed by the reference's compiled code (oracle/_ref), except the inputs.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent
MTX = OUT / "mtx"

MTX_FILES = {
    "general_real.mtx": """%%MatrixMarket matrix coordinate real general
% unsorted entries, empty rows 1 and 5 (0-based), a long row 3, negative values
7 9 17
4 9 -1.5
1 1 2.0
4 1 0.25
4 2 3.0
4 3 -4.0
4 4 5.5
4 5 6.0
4 6 -7.25
4 7 8.0
4 8 9.0
1 9 1e-3
3 2 1.0
7 7 -2.0
7 1 3.0
5 5 1.0
3 8 2.5
1 5 -0.5
""",
    "symmetric_real.mtx": """%%MatrixMarket matrix coordinate real symmetric
5 5 7
1 1 4.0
2 1 -1.0
3 2 -1.0
3 3 4.0
4 3 -1.0
5 1 0.5
5 5 4.0
""",
    "skew_symmetric.mtx": """%%MatrixMarket matrix coordinate real skew-symmetric
4 4 3
2 1 1.5
3 1 -2.0
4 2 3.0
""",
    "pattern_general.mtx": """%%MatrixMarket matrix coordinate pattern general
4 6 6
1 2
1 6
2 1
4 4
4 3
4 5
""",
    "pattern_symmetric.mtx": """%%MatrixMarket matrix coordinate pattern symmetric
4 4 4
1 1
2 1
4 2
4 4
""",
    "integer_general.mtx": """%%MatrixMarket matrix coordinate integer general
3 3 5
1 1 3
1 3 -7
2 2 11
3 1 2
3 3 -1
""",
    "complex_general.mtx": """%%MatrixMarket matrix coordinate complex general
3 4 4
1 1 3.0 4.0
2 4 -1.0 0.0
3 2 0.0 -2.0
3 3 1.0 1.0
""",
    "hermitian.mtx": """%%MatrixMarket matrix coordinate complex Hermitian
3 3 4
1 1 2.0 0.0
2 1 1.0 -1.0
3 2 0.0 3.0
3 3 5.0 0.0
""",
    "duplicates.mtx": """%%MatrixMarket matrix coordinate real general
3 3 6
1 1 1.0
2 2 2.0
1 1 3.0
3 1 4.0
2 2 5.0
3 3 6.0
""",
    "no_header.mtx": """4 4 4
1 1 1.0
2 3 2.0
3 2 3.0
4 4 4.0
""",
}


def write_mtx():
    MTX.mkdir(exist_ok=True)
    for name, text in MTX_FILES.items():
        (MTX / name).write_text(text)


def b_inputs(ncols: int, k: int):
    ones = np.ones(ncols * k, np.float64)
    rnd = O.drand48(42, ncols * k)
    return {"ones": ones, "drand48": rnd}


def make_mtx_fixtures():
    # one OpenMP thread: the reference's row bucketing hands out slots by atomic decrement, so with several threads
    # the order of duplicate (row, col) values depends on thread timing (bucketsort_gen.c:186-194)
    O.ref_lib("d").ref_set_threads(1)
    out = {}
    for name in sorted(MTX_FILES):
        m, n, rp, ci, va = O.ref_mtx_to_csr(str(MTX / name), "d")
        key = name[:-4]
        out[f"{key}.shape"] = np.array([m, n], np.int64)
        out[f"{key}.row_ptr"] = rp
        out[f"{key}.col_idx"] = ci
        out[f"{key}.vals"] = va
        for k in (1, 4, 32):
            for bname, x in b_inputs(n, k).items():
                y = O.ref_spmm(rp, ci, va.copy(), n, x, k)
                out[f"{key}.y.k{k}.{bname}"] = y
    np.savez_compressed(OUT / "mtx_csr.npz", **out)


def make_mtx_f32_fixtures():
    """The fp32 drop-in pin (ValueType=float, make.sh:98-102): per .mtx, the CSR values the reference's FLOAT build
    reads (mtx_read with MATRIX_MARKET_FLOAT_T=float) and C = A*B from its float plugin at K in {1, 4, 32} with
    x = (float) drand48(42) -- the x the fp32 harness / refabi_driver_f hands the plugin."""
    O.ref_lib("f").ref_set_threads(1)
    out = {}
    for name in sorted(MTX_FILES):
        m, n, rp, ci, va = O.ref_mtx_to_csr(str(MTX / name), "f")
        vf = va.astype(np.float32)
        assert np.array_equal(vf.astype(np.float64), va), name          # the float build's values, exactly
        key = name[:-4]
        out[f"{key}.shape"] = np.array([m, n], np.int64)
        out[f"{key}.row_ptr"] = rp
        out[f"{key}.col_idx"] = ci
        out[f"{key}.vals"] = vf
        for k in (1, 4, 32):
            x = O.drand48(42, n * k).astype(np.float32)
            out[f"{key}.y.k{k}.drand48"] = O.ref_spmm(rp, ci, vf.copy(), n, x, k)
    np.savez_compressed(OUT / "mtx_csr_f32.npz", **out)


SMTX = ROOT / "tests" / "golden" / "smtx"


def make_smtx_fixtures():
    """DLMC .smtx inputs (the USE_DLCM_MATRICES path) and the row offsets / columns the reference's smtx_read
    returns (dlcm_matrix.c:258-324; values are time-seeded there, not pinned)."""
    SMTX.mkdir(exist_ok=True)
    rng = np.random.default_rng(21)
    files = {}
    # a transformer-like pruned weight (rows sorted), one with unsorted rows and duplicates, empty rows, one row
    for name, (m, k, dens, shuffle) in {"pruned_64x48": (64, 48, 0.3, False), "unsorted_dups": (40, 30, 0.2, True),
                                        "empty_rows": (25, 60, 0.05, False), "one_row": (1, 17, 0.5, False)}.items():
        deg = rng.binomial(k, dens, m)
        if name == "empty_rows":
            deg[::3] = 0
        rows = []
        for d in deg:
            c = np.sort(rng.choice(k, d, replace=False))
            if shuffle and d > 1:
                c = np.concatenate([c, c[: max(1, d // 4)]])      # duplicates
                rng.shuffle(c)
            rows.append(c)
        rp = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
        ci = np.concatenate(rows).astype(np.int32) if rows else np.zeros(0, np.int32)
        text = f"{m}, {k}, {len(ci)}\n" + " ".join(map(str, rp)) + "\n" + " ".join(map(str, ci)) + "\n"
        files[name] = text
    out = {}
    for name, text in files.items():
        path = SMTX / f"{name}.smtx"
        path.write_text(text)
        m, k, rp, ci = O.ref_smtx_read(str(path))
        out[f"{name}.shape"] = np.array([m, k], np.int64)
        out[f"{name}.row_ptr"] = rp
        out[f"{name}.col_idx"] = ci
    np.savez_compressed(OUT / "smtx_csr.npz", **out)


def random_csr(rng, m, n, mean_deg, long_row=None, empty_frac=0.1):
    deg = rng.poisson(mean_deg, m)
    deg[rng.random(m) < empty_frac] = 0
    deg = np.minimum(deg, n)
    if long_row is not None:
        deg[long_row] = n
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum(deg)
    ci = np.concatenate([np.sort(rng.choice(n, d, replace=False)) for d in deg] or [np.zeros(0)]).astype(np.int32)
    va = rng.uniform(-1.0, 1.0, int(rp[-1]))
    return rp, ci, va


def make_spmm_cases():
    rng = np.random.default_rng(20251015)
    cases = {
        "small": random_csr(rng, 37, 29, 4.0),
        "longrow": random_csr(rng, 300, 257, 6.0, long_row=123),
        "rect_wide": random_csr(rng, 64, 1000, 20.0),
        "rect_tall": random_csr(rng, 900, 50, 3.0, empty_frac=0.3),
        "allempty": (np.zeros(17, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float64)),
    }
    out = {}
    for name, (rp, ci, va) in cases.items():
        m = len(rp) - 1
        n = int(ci.max()) + 1 if len(ci) else 8
        n = max(n, {"small": 29, "longrow": 257, "rect_wide": 1000, "rect_tall": 50}.get(name, 8))
        out[f"{name}.shape"] = np.array([m, n], np.int64)
        out[f"{name}.row_ptr"] = rp
        out[f"{name}.col_idx"] = ci
        out[f"{name}.vals"] = va
        for k in (1, 8, 32, 128):
            if k == 128 and m * k > 10000:
                continue
            x = O.drand48(42 + k, n * k)
            out[f"{name}.x.k{k}"] = x
            out[f"{name}.y_d.k{k}"] = O.ref_spmm(rp, ci, va.copy(), n, x.copy(), k)
            out[f"{name}.y_f.k{k}"] = O.ref_spmm(rp, ci, va.astype(np.float32), n, x.astype(np.float32), k)
    np.savez_compressed(OUT / "spmm_cases.npz", **out)


def make_partition():
    rng = np.random.default_rng(7)
    rps = {}
    d = rng.poisson(5, 1000)
    rps["poisson"] = d
    d = np.zeros(200, np.int64); d[50] = 10000; d[51:] = 1
    rps["one_giant"] = d
    d = rng.poisson(3, 500); d[100:300] = 0
    rps["empty_run"] = d
    rps["uniform"] = np.full(64, 8)
    d = np.zeros(10, np.int64)
    rps["zero_nnz"] = d
    rps["single_row"] = np.array([42])
    out = {}
    for name, deg in rps.items():
        rp = np.zeros(len(deg) + 1, np.int32)
        rp[1:] = np.cumsum(deg)
        nnz = int(rp[-1])
        out[f"{name}.row_ptr"] = rp
        for W in (1, 2, 3, 7, 8, 64, 256):
            b = np.array([O.ref_partition(rp, nnz, W, w) for w in range(W)], np.int64)
            out[f"{name}.W{W}"] = b
    np.savez_compressed(OUT / "partition.npz", **out)


def make_metrics():
    rng = np.random.default_rng(3)
    out = {}
    gold = rng.uniform(-2, 2, 5000)
    pairs = {
        "exact": (gold, gold.copy()),
        "perturbed": (gold, gold * (1 + rng.normal(0, 1e-12, gold.shape))),
        "with_zeros": (np.where(rng.random(5000) < 0.2, 0.0, gold), gold),
        "coarse": (gold, gold.astype(np.float32).astype(np.float64)),
    }
    for name, (g, t) in pairs.items():
        out[f"{name}.gold"] = g
        out[f"{name}.test"] = t
        out[f"{name}.metrics"] = O.ref_metrics(g, t)
    np.savez_compressed(OUT / "metrics.npz", **out)


FEATURE_LINES = ["3000 3000 20 6.6667 normal random 0.3 100 0.95 0.5 14",
                 "5000 4000 5 1.6667 normal random 0.05 0 0.05 0.05 14",
                 "2000 2000 50 16.6667 normal random 0.6 1000 1.4 0.95 14",
                 "1500 1500 100 33.3333 normal random 0.05 10000 1.9 0.5 14",
                 "800 800 200 66.6667 gamma random 0.3 0 0.5 0.05 14",
                 "4000 4000 10 3.3333 normal diagonal 0.3 0 0.95 0.95 14"]
FEATURE_KEYS = ("avg_nnz_per_row", "std_nnz_per_row", "bw", "skew", "avg_num_neighbours", "cross_row_similarity")


def make_features():
    sys.path.insert(0, str(ROOT / "spmm-research_amd"))
    import spmm_amd as S
    out, names = {}, []
    pats = {}
    for f in sorted(MTX.glob("*.mtx")):
        M, n, rp, ci, _ = O.ref_mtx_to_csr(str(f))
        if M > 0 and len(ci) > 0:
            pats[f.stem] = (rp, ci, n)
    rng = np.random.default_rng(11)
    for t in range(4):   # random sorted rows incl. empty ones and duplicates-free runs
        m, n = 300 + 100 * t, 700
        rows = [np.unique(rng.integers(0, n, rng.integers(0, 30))) if rng.random() > 0.2 else np.zeros(0, int)
                for _ in range(m)]
        rp = np.zeros(m + 1, np.int32)
        rp[1:] = np.cumsum([len(r) for r in rows])
        pats[f"random{t}"] = (rp, np.concatenate(rows).astype(np.int32), n)
    for q, line in enumerate(FEATURE_LINES):
        A = S.generate(S.gen_params(line))
        pats[f"gen{q}"] = (A.row_ptr, A.col_idx, A.ncols)
    for name, (rp, ci, n) in pats.items():
        r = O.ref_features(rp, ci, n)
        out[f"{name}.row_ptr"] = np.asarray(rp, np.int32)
        out[f"{name}.col_idx"] = np.asarray(ci, np.int32)
        out[f"{name}.ncols"] = np.int64(n)
        out[f"{name}.features"] = np.array([r[k] for k in FEATURE_KEYS], np.float64)
        names.append(name)
    out["keys"] = np.array(FEATURE_KEYS)
    np.savez_compressed(OUT / "features.npz", **out)


def main():
    if not O.ref_available("d"):
        raise SystemExit("oracle/_ref not built: run `make -C oracle` in a container with /root/reference")
    only = sys.argv[1:]
    if only:                       # e.g. `make_golden.py make_mtx_f32_fixtures`: regenerate named fixtures only
        for fn in only:
            globals()[fn]()
        return
    write_mtx()
    make_mtx_fixtures()
    make_mtx_f32_fixtures()
    make_smtx_fixtures()
    make_spmm_cases()
    make_partition()
    make_metrics()
    make_features()
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
