"""The perfect-balance K = 1 format (include/spmm_pbv.h) on the GPU against the oracle, -m gpu.

Parity contract (include/spmm_pbv.h): rows the format reports exact (all items in one lane) are BIT-IDENTICAL to the
oracle's restatement of the reference's serial row (spmm_kernel_csr.cpp:70-96 at K = 1); every row is within 1e-10
normwise of the __float128 gold (fp64) or (n+1)*2^-24 (fp32).  Cases: generator lines of the medium dataset's
classes, a skewed (gamma, 10^4) line, long runs of empty rows, one row spanning many blocks, nnz = 0, m = 1, E in
{4, 8, 16}, both dtypes; run-to-run determinism; the host entry point at K > 1 (one SpMV per column of x) and the
strided device entry point; the reference-header plugin on the reference's golden .mtx fixtures.
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from gpu_check import check_rows

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
LINES = {
    "avg5_bw06": "60000 60000 5 1.6667 normal random 0.6 100 0.5 0.95 14",
    "avg20_bw03": "200000 200000 20 6.6667 normal random 0.3 100 0.95 0.5 14",
    "avg500_bw005": "8000 8000 500 166.6667 normal random 0.05 100 0.95 0.95 14",
    "gamma_skew": "60000 60000 50 16.6667 gamma random 0.3 10000 0.95 0.5 14",
}


@pytest.fixture(scope="module")
def env():
    import torch
    import spmm_amd as S
    import spmm_amd.pbv as P
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, S, P, O


def _csr(S, rp, ci, vals, ncols):
    return S.CSR(np.asarray(rp, np.int32), np.asarray(ci, np.int32), np.asarray(vals, np.float64), len(rp) - 1, ncols)


def run_pbv(torch, P, A, e, dtype=np.float64, seed=5, ldy=1):
    dev = torch.device("cuda", 0)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.rand(max(A.ncols, 1), generator=g, device=dev, dtype=tdt)
    y = torch.full((max(A.m, 1), ldy), float("nan"), device=dev, dtype=tdt)
    f = P.PBVFormat(A.row_ptr, A.col_idx, A.values.astype(dtype), A.m, A.ncols, A.nnz, 0, e)
    f.spmv_device(x.data_ptr(), y.data_ptr(), ldy, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ex, inf = f.exact_rows(), f.info()
    f.close()
    return x.cpu().numpy().reshape(-1, 1), y.cpu().numpy()[:A.m], ex, inf


def check_all(O, A, x, y, ex, dtype=np.float64):
    rows = np.arange(A.m)
    for c in range(0, A.m, 50000):        # the oracle per chunk of rows (sub-CSR with renumbered columns)
        check_rows(O, A, x, y, ex, rows[c:c + 50000], dtype)


@pytest.mark.parametrize("e", [4, 8, 16])
@pytest.mark.parametrize("name", list(LINES))
def test_generator_lines(env, name, e):
    torch, S, P, O = env
    A = S.generate(S.gen_params(LINES[name]))
    x, y, ex, inf = run_pbv(torch, P, A, e)
    assert inf["exact_rows"] == int(ex.sum()) and inf["items_per_lane"] == e
    check_all(O, A, x, y, ex)
    # deterministic run to run
    _, y2, _, _ = run_pbv(torch, P, A, e)
    assert np.array_equal(y.view(np.int64), y2.view(np.int64))


@pytest.mark.parametrize("name", ["avg20_bw03", "gamma_skew"])
def test_fp32(env, name):
    torch, S, P, O = env
    A = S.generate(S.gen_params(LINES[name]))
    x, y, ex, _ = run_pbv(torch, P, A, 8, np.float32)
    check_all(O, A, x.astype(np.float32), y, ex, np.float32)


def test_structural_edge_cases(env):
    torch, S, P, O = env
    rng = np.random.default_rng(3)
    cases = []
    # long runs of empty rows (more row ends than one block holds) between dense rows
    deg = np.where(rng.random(30000) < 0.01, rng.integers(100, 3000, 30000), 0)
    cases.append(deg)
    # one row of 200,000 nonzeros (dozens of blocks) between short rows, and a last row that is empty
    deg = rng.integers(0, 6, 5000)
    deg[2500] = 200000
    deg[-1] = 0
    cases.append(deg)
    # single row; all rows empty
    cases.append(np.array([777]))
    cases.append(np.zeros(70000, np.int64))
    for deg in cases:
        rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
        ncols = 4096
        ci = np.concatenate([np.sort(rng.choice(ncols, int(d), replace=int(d) > ncols)) for d in deg]) \
            if rp[-1] else np.zeros(0, np.int32)
        A = _csr(S, rp, ci, rng.standard_normal(int(rp[-1])), ncols)
        for e in (4, 16):
            x, y, ex, inf = run_pbv(torch, P, A, e)
            check_all(O, A, x, y, ex)
            if A.nnz == 0:
                assert ex.all() and (y == 0).all()


def test_host_run_k_columns_and_strided_device(env):
    torch, S, P, O = env
    A = S.generate(S.gen_params(LINES["gamma_skew"]))
    k = 4
    xk = O.drand48(42, A.ncols * k)                  # reference layout: column-major [k][ncols]
    f = P.PBVFormat(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz)
    y = np.zeros(A.m * k)
    f.spmm(xk, y, k)
    Y = y.reshape(A.m, k)
    ex = f.exact_rows()
    for c in range(k):                               # column c equals the single-vector device run on x column c
        xd = torch.from_numpy(xk[c * A.ncols:(c + 1) * A.ncols].copy()).cuda()
        yd = torch.full((A.m, 3), float("nan"), dtype=torch.float64, device="cuda")
        f.spmv_device(xd.data_ptr(), yd[:, 1:].data_ptr(), 3, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        yc = yd.cpu().numpy()
        assert np.isnan(yc[:, 0]).all() and np.isnan(yc[:, 2]).all()     # ldy = 3: only column 1 written
        assert np.array_equal(yc[:, 1].view(np.int64), Y[:, c].view(np.int64))
    Bh = np.ascontiguousarray(xk.reshape(k, A.ncols).T)
    check_rows(O, A, Bh, Y, ex, np.arange(0, A.m, 7))
    assert f.last_ms() > 0
    stats = f.statistics_print_data().split(",")
    assert len(stats) == 9 and int(stats[5]) == f.info()["blocks"]
    f.close()


@pytest.mark.parametrize("vt", ["d", "f"])
def test_reference_plugin_pbv(golden, tmp_path, vt):
    """integration/spmm_kernel_hip_pbv.cpp, compiled against the reference's spmv_kernel.h, on the golden .mtx files
    at K = 1: exact rows equal the reference's own outputs bit for bit, the rest within the normwise bound."""
    import spmm_amd as S
    import spmm_amd.pbv as P
    exe = ROOT / "integration" / "bin" / f"refabi_pbv_{vt}.exe"
    assert exe.exists(), f"{exe} missing: run make -C integration"
    g = golden("mtx_csr.npz" if vt == "d" else "mtx_csr_f32.npz")
    dt = np.float64 if vt == "d" else np.float32
    it = np.int64 if vt == "d" else np.int32
    n = 0
    for path in sorted((ROOT / "tests" / "golden" / "mtx").glob("*.mtx")):
        name = path.stem
        key = f"{name}.y.k1.drand48"
        if key not in g:
            continue
        out = tmp_path / f"{name}.bin"
        r = subprocess.run([str(exe), str(path), "1", str(out)], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, SPMM_PBV_ITEMS="4"))
        assert r.returncode == 0, r.stderr
        A, _, _ = S.mtx_read(path)
        _, ex = P.plan_host(A.row_ptr, A.m, A.nnz, 4)
        y = np.fromfile(out, dt)
        want = g[key].reshape(-1)
        assert np.array_equal(y[ex].view(it), want[ex].view(it)), name
        # split rows: |y - reference| <= 2 x the normwise bound (each is within it of the exact sum), |A||x| scale
        x = S.drand48(42, A.ncols).astype(dt).astype(np.float64)
        deg = np.diff(A.row_ptr)
        rows = np.repeat(np.arange(A.m), deg)
        absdot = np.bincount(rows, weights=np.abs(A.values.astype(dt).astype(np.float64)) * np.abs(x[A.col_idx]),
                             minlength=A.m)
        tol = 1e-10 if vt == "d" else (deg + 1) * 2.0 ** -24 * 1.01
        err = np.abs(y.astype(np.float64) - want.astype(np.float64))
        assert (err[~ex] <= 2 * (tol if np.isscalar(tol) else tol[~ex]) * np.maximum(np.abs(want[~ex]), absdot[~ex])
                ).all(), name
        n += 1
    assert n >= 5
