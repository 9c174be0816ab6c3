"""GPU parity of the sparse-attention pipeline consumer against the oracle restatement.

Stages (reference compute() step, pipeline_code_bench/sddmm_bench.cpp:918-937):
  K/Q/V = W x         engine SpMM, row-major x: rows the engine reports exact are bit-identical to the oracle chain
  y = SDDMM           spmm_sddmm: bit-identical to oracle_sddmm (one FMA chain over n, then x mask value), for the
                      reference's row-i-of-K product (mode 0) and Q K^T (mode 1)
  softmax (optional)  within 1e-12 (fp64) / 1e-5 (fp32) relative of the serial reference order
  y_final = mask(y) V engine SpMM with the SDDMM output as values (spmm_hip_update_values[_device])
Also: host path == device path, a hipGraph replay, value updates under tiles / windows, and the reference-side
plugin (integration/refpipe_driver) driven like the reference harness.
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


EXACT = {"SPMM_HIP_SEQ_MAX": "2048", "SPMM_HIP_LANES": "-1"}    # every row one FMA chain (rows here < 2048)


@pytest.fixture
def env(monkeypatch):
    for kk, vv in EXACT.items():
        monkeypatch.setenv(kk, vv)
    import torch
    import spmm_amd as S
    from spmm_amd import pipeline as P
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, S, P, O


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64 if a.dtype == np.float64 else np.int32)


def make(P, m=256, k=192, n=64, wd=0.3, md=0.1, band=8, seed=0):
    w = [P.dlmc_like_weight(m, k, wd, seed + i) for i in range(3)]
    mask = P.band_and_random_mask(m, md, band, seed + 7)
    x = np.random.default_rng(seed + 11).uniform(0, 1, (k, n))
    return w, mask, x


def oracle_pipeline(O, w, mask, x, dtype, mode, softmax=False):
    x = x.astype(dtype)
    K, Q, V = (O.spmm_rowmajor(a.row_ptr, a.col_idx, a.values.astype(dtype), a.ncols, x) for a in w)
    y = O.sddmm(mask.row_ptr, mask.col_idx, mask.values.astype(dtype), Q, K, mode)
    if softmax:
        y = O.softmax(y)
    return K, Q, V, y


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("mode", [0, 1])
def test_pipeline_stages_bitexact(env, dtype, mode):
    torch, S, P, O = env
    w, mask, x = make(P)
    pipe = P.SparseAttentionPipeline(*w, mask, x.shape[1], dtype, mode)
    out = pipe.run(x)
    K, Q, V, y = oracle_pipeline(O, w, mask, x, dtype, mode)
    for t, want in (("K", K), ("Q", Q), ("V", V)):
        ex = pipe.mf[t].exact_rows()
        assert ex.all()
        assert np.array_equal(bits(out[t]), bits(want)), t
    assert np.array_equal(bits(out["y"]), bits(y))
    # final SpMM on the GPU's own y (the mask pattern with the SDDMM values): the oracle chain, bit for bit
    yf = O.spmm_rowmajor(mask.row_ptr, mask.col_idx, out["y"], mask.ncols, out["V"])
    ex = pipe.final.exact_rows()
    assert np.array_equal(bits(out["y_final"][ex]), bits(yf[ex]))
    pipe.close()


@pytest.mark.parametrize("dtype,rtol", [(np.float64, 1e-12), (np.float32, 2e-5)])
def test_pipeline_softmax(env, dtype, rtol):
    torch, S, P, O = env
    w, mask, x = make(P, m=200, k=128, n=32, seed=3)
    x = x * 0.05                                             # keep exp() in range: scores ~ O(1)
    pipe = P.SparseAttentionPipeline(*w, mask, x.shape[1], dtype, P.SDDMM_QKT | P.SDDMM_SOFTMAX)
    out = pipe.run(x)
    K, Q, V, y = oracle_pipeline(O, w, mask, x, dtype, 1, softmax=True)
    assert np.allclose(out["y"], y, rtol=rtol, atol=0)
    assert abs(float(out["y"].astype(np.float64).sum()) - 1.0) < (1e-12 if dtype == np.float64 else 1e-4)
    pipe.close()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_pipeline_device_path_and_graph(env, dtype):
    """run_device (HBM-resident, stream-ordered) == the host path bit for bit; one step captured in a hipGraph and
    replayed gives the same bits."""
    torch, S, P, O = env
    w, mask, x = make(P, m=320, k=256, n=64, seed=5)
    pipe = P.SparseAttentionPipeline(*w, mask, x.shape[1], dtype, 0)
    host = pipe.run(x)
    dev = torch.device("cuda", 0)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    n = x.shape[1]
    bx = torch.from_numpy(x.astype(dtype)).to(dev)
    bufs = {t: torch.zeros((a.m, n), dtype=tdt, device=dev) for t, a in zip("KQV", w)}
    y = torch.zeros(mask.nnz, dtype=tdt, device=dev)
    out = torch.zeros((mask.m, n), dtype=tdt, device=dev)
    s = torch.cuda.Stream(dev)
    args = (bx.data_ptr(), bufs["K"].data_ptr(), bufs["Q"].data_ptr(), bufs["V"].data_ptr(), y.data_ptr(),
            out.data_ptr())
    with torch.cuda.stream(s):
        pipe.run_device(*args, s.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(host["y_final"]))
    assert np.array_equal(bits(y.cpu().numpy()), bits(host["y"]))
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pipe.run_device(*args, s.cuda_stream)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(host["y_final"]))
    pipe.close()


@pytest.mark.parametrize("force", [{"SPMM_HIP_TILES": "1"}, {"SPMM_HIP_TILES": "1", "SPMM_HIP_MFMA": "-1"},
                                   {"SPMM_HIP_WIN_BYTES": "4096"}, {}])
def test_update_values_regathers(env, monkeypatch, force):
    """New values through spmm_hip_update_values[_device] == a handle built with them, also when the plan keeps
    window-major (chained) or tile (chunk-major) copies of the values."""
    torch, S, P, O = env
    for kk in EXACT:
        monkeypatch.delenv(kk)
    for kk, vv in force.items():
        monkeypatch.setenv(kk, vv)
    A = S.generate(S.gen_params("4000 4000 40 13 normal random 0.1 0 0.95 0.95 14"))
    k = 32
    x = O.drand48(3, A.ncols * k)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    if "SPMM_HIP_TILES" in force:
        assert mf.tile_info()["tiles"] > 0
    if "SPMM_HIP_WIN_BYTES" in force:
        assert mf.info()[12] > 1
    v2 = np.random.default_rng(9).uniform(-1, 1, A.nnz)
    mf.update_values(v2)
    y = np.zeros(A.m * k)
    mf.spmm(x, y, k)
    ex = mf.exact_rows()
    want = O.spmm(A.row_ptr, A.col_idx, v2, A.ncols, x, k)
    assert np.array_equal(bits(y.reshape(A.m, k)[ex]), bits(want[ex]))
    # device variant
    dev = torch.device("cuda", 0)
    v3 = torch.from_numpy(np.random.default_rng(10).uniform(-1, 1, A.nnz)).to(dev)
    mf.update_values_device(v3.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    mf.spmm(x, y, k)
    want = O.spmm(A.row_ptr, A.col_idx, v3.cpu().numpy(), A.ncols, x, k)
    assert np.array_equal(bits(y.reshape(A.m, k)[ex]), bits(want[ex]))
    mf.close()


def _write_inputs(path, w, mask, x, dtype):
    with open(path, "wb") as f:
        np.array([x.shape[1]], np.int64).tofile(f)
        for a in list(w) + [mask]:
            np.array([a.m, a.ncols, a.nnz], np.int64).tofile(f)
            a.row_ptr.astype(np.int32).tofile(f)
            a.col_idx.astype(np.int32).tofile(f)
            a.values.astype(dtype).tofile(f)
        x.astype(dtype).tofile(f)


@pytest.mark.parametrize("vt,dtype", [("d", np.float64), ("f", np.float32)])
@pytest.mark.parametrize("mode", [0, 1])
def test_reference_plugin_pipeline(env, tmp_path, vt, dtype, mode):
    """integration/sddmm_kernel_hip.cpp (compiled against the reference's sddmm_kernel.h) driven like compute()."""
    torch, S, P, O = env
    exe = ROOT / "integration" / "bin" / f"refpipe_driver_{vt}.exe"
    assert exe.exists(), "run make -C integration"
    w, mask, x = make(P, m=192, k=160, n=48, seed=8)
    _write_inputs(tmp_path / "in.bin", w, mask, x, dtype)
    r = subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, SPMM_SDDMM_MODE=str(mode), **EXACT))
    assert r.returncode == 0, r.stderr
    assert "HIP_SDDMM_PIPELINE_MI355X" in r.stdout
    raw = np.fromfile(tmp_path / "out.bin", dtype)
    n = x.shape[1]
    sizes = [a.m * n for a in w] + [mask.nnz, mask.m * n]
    parts = np.split(raw, np.cumsum(sizes)[:-1])
    K, Q, V, y = oracle_pipeline(O, w, mask, x, dtype, mode)
    for got, want in zip(parts[:4], (K, Q, V, y)):
        assert np.array_equal(bits(got), bits(want.ravel()))
    yf = O.spmm_rowmajor(mask.row_ptr, mask.col_idx, parts[3], mask.ncols, parts[2].reshape(-1, n))
    assert np.array_equal(bits(parts[4]), bits(yf.ravel()))


def test_run_device_batch_equals_sequential(env, monkeypatch):
    """spmm_hip_run_device_batch (independent handles on forked side streams) == one spmm_hip_run_device per handle,
    bit for bit, eagerly and replayed from a captured hipGraph; split rows allowed (default inspector)."""
    torch, S, P, O = env
    monkeypatch.delenv("SPMM_HIP_SEQ_MAX")
    monkeypatch.delenv("SPMM_HIP_LANES")
    dev = torch.device("cuda", 0)
    mats = [S.generate(S.gen_params(l)) for l in ("3000 2000 40 30 normal random 0.3 1000 0.5 0.5 14",
                                                  "5000 2000 8 2 normal random 0.05 0 0.5 0.95 14",
                                                  "700 2000 300 100 normal random 0.6 10 0.5 0.5 14")]
    k = 48
    mfs = [S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0) for A in mats]
    B = torch.rand((2000, k), dtype=torch.float64, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    Bt = B.t().contiguous()                                   # the same B column-major for the second entry
    lay = [S.B_ROW_MAJOR, S.B_COL_MAJOR, S.B_ROW_MAJOR]
    bsrc = [B, Bt, B]
    want, got = [], []
    s = torch.cuda.Stream(dev)
    for mf, A, b, L in zip(mfs, mats, bsrc, lay):
        c = torch.empty((A.m, k), dtype=torch.float64, device=dev)
        with torch.cuda.stream(s):
            mf.spmm_device(b.data_ptr(), L, c.data_ptr(), k, s.cuda_stream)
        want.append(c)
        got.append(torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev))
    entries = [(mf, b.data_ptr(), L, c.data_ptr(), k) for mf, b, L, c in zip(mfs, bsrc, lay, got)]
    with torch.cuda.stream(s):
        S.run_device_batch(entries, s.cuda_stream)
    torch.cuda.synchronize()
    for w, g in zip(want, got):
        assert np.array_equal(bits(w.cpu().numpy()), bits(g.cpu().numpy()))
    for g in got:
        g.fill_(float("nan"))
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        S.run_device_batch(entries, s.cuda_stream)
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    for w, g in zip(want, got):
        assert np.array_equal(bits(w.cpu().numpy()), bits(g.cpu().numpy()))
    for mf in mfs:
        mf.close()
