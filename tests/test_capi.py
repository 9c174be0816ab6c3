"""The C-ABI libraries load without a GPU and export every function the include/*.h headers declare."""
import ctypes
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "spmm-research_amd" / "lib"


def declared(header: str) -> list[str]:
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(spmm_(?:hip|host|sddmm|pbv)_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("header,lib", [("spmm_hip.h", "libspmm_hip.so"), ("spmm_host.h", "libspmm_host.so"),
                                        ("spmm_pipeline.h", "libspmm_hip.so"), ("spmm_pbv.h", "libspmm_pbv.so")])
def test_exports_every_declared_symbol(header, lib):
    names = declared(header)
    assert len(names) >= (4 if header == "spmm_pipeline.h" else 10)
    L = ctypes.CDLL(str(LIB / lib))
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and they are plain C symbols (not C++-mangled)
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB / lib)], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", out, re.M), n


def test_host_only_entry_points_without_gpu():
    import spmm_amd as S
    assert S.hip.spmm_hip_strerror(-6) == b"malformed CSR"
    assert S.stats_labels().startswith(",kernel_ms")
    # the gfx950 code object is embedded (offload bundle id)
    assert b"amdgcn-amd-amdhsa--gfx950" in (LIB / "libspmm_hip.so").read_bytes()


def test_harness_prints_reference_labels():
    exe = ROOT / "spmm-research_amd" / "bin" / "spmm_csr_hip_d.exe"
    r = subprocess.run([str(exe)], capture_output=True, text=True, env={"NUM_COLS": "32"})
    assert r.returncode == 0
    labels = r.stderr.strip().split(",")
    assert labels[:12] == ["matrix_name", "num_threads", "input_columns", "csr_m", "csr_k", "csr_nnz", "time",
                           "gflops", "csr_mem_footprint", "m", "n", "nnz"]
    assert "kernel_ms" in labels and "roofline_frac" in labels
    r = subprocess.run([str(exe)], capture_output=True, text=True, env={"USE_ARTIFICIAL_MATRICES": "1"})
    assert r.stderr.startswith("matrix_name,distribution,placement,seed,nr_rows")


def test_single_hip_runtime_in_process():
    """Importing the engine before torch must not leave two HIP runtimes mapped (spmm_amd preloads torch's)."""
    code = ("import sys; sys.path.insert(0, 'spmm-research_amd'); import spmm_amd, torch; "
            "maps = open('/proc/self/maps').read(); "
            "print(len({l.split()[-1] for l in maps.splitlines() if 'libamdhip64' in l}))")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "1"


def test_multi_gpu_factory_fails_loudly_without_gpu():
    """spmm_hip_create_multi validates its arguments, then needs devices: no CPU fallback."""
    import numpy as np
    import spmm_amd as S
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible: tests/test_gpu_multi.py covers the multi-GPU handle")
    except ImportError:
        pass
    rp = np.array([0, 1, 2], np.int32)
    ci = np.array([0, 1], np.int32)
    va = np.ones(2)
    with pytest.raises(S.SpmmHipError) as e:
        S.csr_to_format(rp, ci, va, 2, 2, 2, 4, ngpus=2)
    assert e.value.status == -4                              # no HIP device
    h = ctypes.c_void_p()
    assert S.hip.spmm_hip_create_multi(rp, ci, va.ctypes.data_as(ctypes.c_void_p), 2, 2, 2, 4, 0, 0, None,
                                       ctypes.byref(h)) == -1        # ngpus < 1
    bad = np.array([0, 2, 1], np.int32)
    assert S.hip.spmm_hip_create_multi(bad, ci, va.ctypes.data_as(ctypes.c_void_p), 2, 2, 1, 4, 0, 2, None,
                                       ctypes.byref(h)) == -6        # malformed CSR (before any device work)


@pytest.mark.parametrize("lib", ["libspmm_hip.so", "libspmm_pbv.so"])
def test_device_code_holds_every_registered_kernel(lib):
    """Every kernel the host half registers is in the library's gfx950 code objects (tools/check_fatbin.py): a device
    half compiled from an older source than its host half would load and abort at the first launch."""
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "check_fatbin.py"), str(LIB / lib)], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "missing 0" in r.stdout
