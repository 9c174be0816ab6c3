"""Multi-GPU handles in the C ABI (SURVEY §8b `ngpus`; include/spmm_hip.h spmm_hip_create_multi), -m gpu.

The box has one GPU, so every shard is mapped onto device 0 (the test mode of the path: the same partition, per-shard
plans, B replication by peer copies and C gathers, just all on one device).  A multi handle's rows are exactly the
rows one single-device handle computes over the same row range, so:
  * against ONE whole-matrix handle: bit-equal on every row both compute exactly (>= 99 % of rows), normwise 1e-10
    elsewhere, and bit-equal to the oracle on the rows the multi handle reports exact;
  * every entry point (host run, row-major host run, device run into a root-device C, broadcast_b + run_sharded with
    C left in the shards) gives the same bits;
  * the reference-ABI plugin (integration/bin/refabi_driver_d.exe, built against the reference's spmv_kernel.h) with
    SPMM_HIP_NGPUS=4 SPMM_HIP_DEVICES=0,0,0,0 reproduces the reference's golden C bit for bit.
The RCCL broadcast mode (SPMM_HIP_BCAST=rccl) needs distinct devices; on one GPU it runs with one shard.
"""
import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from gpu_check import check_rows, sample_rows

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
LINES = ["200000 200000 20 6.6667 normal random 0.3 100 0.95 0.5 14",
         "60000 60000 50 16.6667 gamma random 0.3 10000 0.95 0.5 14"]      # skewed: split rows in some shards


@pytest.fixture(scope="module")
def env():
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, S, O


def _d2h(ptr: int, nbytes: int, dtype) -> np.ndarray:
    """Copy a raw device buffer (a shard's C) to the host through the HIP runtime the process already uses."""
    import torch
    rt = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype)
    rt.hipDeviceSynchronize()
    assert rt.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0
    return out


@pytest.mark.parametrize("line", LINES, ids=["config2_shape", "gamma_skew"])
@pytest.mark.parametrize("k", [8, 32])
def test_multi_handle_four_shards_on_one_gpu(env, line, k):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    x = O.drand48(42, A.ncols * k)                         # reference layout: column-major B
    one = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    y1 = np.zeros(A.m * k)
    one.spmm(x, y1, k)
    ex1 = one.exact_rows()
    one.close()
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, devices=[0, 0, 0, 0])
    assert mf.ngpus() == (4, 0)
    sh = [mf.shard(g) for g in range(4)]
    assert sh[0]["row0"] == 0 and sh[-1]["row1"] == A.m
    for g in range(4):
        assert (sh[g]["row0"], sh[g]["row1"]) == O.partition(A.row_ptr, A.nnz, 4, g)
    ex = mf.exact_rows()
    assert ex.mean() > 0.99 and (ex & ex1).mean() > 0.99
    # host path (the reference contract: x column-major, y row-major, synchronous)
    y = np.zeros(A.m * k)
    mf.spmm(x, y, k)
    Y, Y1 = y.reshape(A.m, k), y1.reshape(A.m, k)
    both = ex & ex1
    assert np.array_equal(Y[both].view(np.int64), Y1[both].view(np.int64))
    Bh = np.ascontiguousarray(x.reshape(k, A.ncols).T)
    check_rows(O, A, Bh, Y, ex, sample_rows(A, 1500))
    assert np.isfinite(Y).all()
    # row-major host path
    yr = np.zeros(A.m * k)
    mf.spmm_rowmajor(np.ascontiguousarray(Bh).ravel(), yr, k)
    assert np.array_equal(yr.view(np.int64), y.view(np.int64))
    # device path: B and C on the root device; both B layouts
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for layout, Bd in ((S.B_ROW_MAJOR, torch.from_numpy(Bh).to(dev)), (S.B_COL_MAJOR, torch.from_numpy(x).to(dev))):
        Cd = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
        mf.spmm_device(Bd.data_ptr(), layout, Cd.data_ptr(), k, s)
        torch.cuda.synchronize()
        assert np.array_equal(Cd.cpu().numpy().view(np.int64), Y.view(np.int64)), layout
    # the timed path: B replicated once, C left sharded
    mf.broadcast_b(torch.from_numpy(Bh).to(dev).data_ptr(), S.B_ROW_MAJOR, k, s)
    mf.run_sharded(k, s)
    torch.cuda.synchronize()
    for g in range(4):
        r0, r1 = sh[g]["row0"], sh[g]["row1"]
        c = _d2h(mf.shard(g)["d_c"], (r1 - r0) * k * 8, np.float64).reshape(r1 - r0, k)
        assert np.array_equal(c.view(np.int64), Y[r0:r1].view(np.int64)), g
    stats = mf.statistics_print_data()
    assert stats.endswith(",4")                             # ngpus column
    mf.close()


def test_multi_handle_fp32_and_value_update(env):
    torch, S, O = env
    A = S.generate(S.gen_params(LINES[0]))
    k = 32
    vals = A.values.astype(np.float32)
    x = O.drand48(42, A.ncols * k).astype(np.float32)
    one = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
    mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, devices=[0, 0, 0])
    for v in (vals, (vals * 0.5 + 0.25).astype(np.float32)):
        one.update_values(v)
        mf.update_values(v)
        y1, y = np.zeros(A.m * k, np.float32), np.zeros(A.m * k, np.float32)
        one.spmm(x, y1, k)
        mf.spmm(x, y, k)
        both = np.repeat(one.exact_rows() & mf.exact_rows(), k)
        assert both.mean() > 0.99
        assert np.array_equal(y[both].view(np.int32), y1[both].view(np.int32))
    one.close()
    mf.close()


def test_multi_handle_rccl_broadcast_one_shard(env, monkeypatch):
    """SPMM_HIP_BCAST=rccl: B replicated by an RCCL broadcast over the shards' communicator (one rank on one GPU)."""
    torch, S, O = env
    A = S.generate(S.gen_params(LINES[0]))
    k = 32
    x = O.drand48(42, A.ncols * k)
    one = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    y1 = np.zeros(A.m * k)
    one.spmm(x, y1, k)
    one.close()
    monkeypatch.setenv("SPMM_HIP_BCAST", "rccl")
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, devices=[0])
    assert mf.ngpus() == (1, 1)
    y = np.zeros(A.m * k)
    mf.spmm(x, y, k)
    mf.close()
    assert np.array_equal(y.view(np.int64), y1.view(np.int64))
    with pytest.raises(S.SpmmHipError):                    # one RCCL rank per GPU: repeated devices are refused
        S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, devices=[0, 0])


@pytest.mark.parametrize("k", [1, 4, 32])
def test_reference_plugin_multi_gpu_bitexact(golden, tmp_path, k):
    exe = ROOT / "integration" / "bin" / "refabi_driver_d.exe"
    assert exe.exists(), "integration/bin/refabi_driver_d.exe missing: run make -C integration"
    g = golden("mtx_csr.npz")
    env = dict(os.environ, SPMM_HIP_NGPUS="4", SPMM_HIP_DEVICES="0,0,0,0")
    for path in sorted((ROOT / "tests" / "golden" / "mtx").glob("*.mtx")):
        name = path.stem
        out = tmp_path / f"{name}.{k}.bin"
        r = subprocess.run([str(exe), str(path), str(k), str(out)], capture_output=True, text=True, timeout=120,
                           env=env)
        assert r.returncode == 0, r.stderr
        assert r.stdout.rstrip().split("\n")[-1].endswith(",4")            # stats: ngpus column
        m = int(g[f"{name}.shape"][0])
        y = np.fromfile(out, np.float64).reshape(m, k)
        want = g[f"{name}.y.k{k}.drand48"]
        assert np.array_equal(y.view(np.int64), want.view(np.int64)), name
