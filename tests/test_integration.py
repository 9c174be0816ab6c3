"""The reference-side plugin (INTEGRATION.md §1 = integration/spmm_kernel_hip.cpp) against the REFERENCE's header.

* CPU: integration/Makefile compiles the plugin and a harness-like driver against
  /root/reference/benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h (+ spmv_bench_common.h, macros/cpp_defines.h)
  with the reference flags (make.sh:39-102) and links them to libspmm_hip.so; nothing of the reference's code ends
  up in the binary (its headers only declare); without a GPU the plugin takes the reference's fatal path
  (exit(EXIT_FAILURE), lib/debug.h:117,127).
* GPU: the driver runs csr_to_format -> MF->spmm(x, y, K) (spmv_bench.cpp:996,318,372) on every golden .mtx at
  K in {1, 4, 32} with x = drand48(42) column-major; y must equal the reference plugin's golden output bit for bit.
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
INTEG = ROOT / "integration"
REF_HDR = Path("/root/reference/benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h")
MTX = sorted((ROOT / "tests" / "golden" / "mtx").glob("*.mtx"))


def _exe(vt):
    return INTEG / "bin" / f"refabi_driver_{vt}.exe"


@pytest.mark.skipif(not REF_HDR.exists(), reason="reference tree absent (the GPU box uses the prebuilt driver)")
def test_plugin_builds_against_reference_header():
    r = subprocess.run(["make", "-C", str(INTEG), "-B"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "error" not in r.stderr.lower()
    for vt in ("d", "f"):
        syms = subprocess.run(["nm", "-C", "--defined-only", str(_exe(vt))], capture_output=True, text=True).stdout
        assert "csr_to_format" in syms and "HipCSR::spmm" in syms
        assert "val_to_double" not in syms           # the reference header's only function body is not emitted


@pytest.mark.skipif(not _exe("d").exists(), reason="integration driver not built")
def test_plugin_fatal_path_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible: the GPU test covers the plugin")
    except ImportError:
        pass
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([str(_exe("d")), str(MTX[0]), "4", os.devnull], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 1
    assert "spmm_hip_create" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 4, 32])
def test_plugin_drives_engine_bitexact(golden, tmp_path, k):
    assert _exe("d").exists(), "integration/bin/refabi_driver_d.exe missing: run make -C integration"
    g = golden("mtx_csr.npz")
    for path in MTX:
        name = path.stem
        out = tmp_path / f"{name}.{k}.bin"
        r = subprocess.run([str(_exe("d")), str(path), str(k), str(out)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "format_name=HIP_CSR_MI355X" in r.stdout
        m = int(g[f"{name}.shape"][0])
        y = np.fromfile(out, np.float64).reshape(m, k)
        want = g[f"{name}.y.k{k}.drand48"]
        assert np.array_equal(y.view(np.int64), want.view(np.int64)), name


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 4, 32])
def test_plugin_f32_drives_engine_bitexact(golden, tmp_path, k):
    """The fp32 drop-in (refabi_driver_f = the plugin compiled with ValueType=float) against the reference's own
    FLOAT build (mtx_csr_f32.npz, tests/golden/make_golden.py): bit for bit."""
    assert _exe("f").exists()
    g = golden("mtx_csr_f32.npz")
    for path in MTX:
        name = path.stem
        out = tmp_path / f"{name}.{k}.bin"
        r = subprocess.run([str(_exe("f")), str(path), str(k), str(out)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        m = int(g[f"{name}.shape"][0])
        y = np.fromfile(out, np.float32).reshape(m, k)
        want = g[f"{name}.y.k{k}.drand48"]
        assert want.dtype == np.float32
        assert np.array_equal(y.view(np.int32), want.view(np.int32)), name
