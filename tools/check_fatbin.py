#!/usr/bin/env python3
"""tools/check_fatbin.py -- every __global__ kernel a library's host code registers is present in its gfx950 device
code object.  (A device object compiled from an older source than its host half -- two hipcc runs of one source at
once -- loads fine and aborts at the first launch: "Cannot find Symbol with name ...".)

  python tools/check_fatbin.py spmm-research_amd/lib/libspmm_hip.so [...]      exit 1 on a missing kernel
"""
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/llvm/bin")


def device_symbols(lib: Path) -> set:
    """Kernel symbols of every gfx950 code object in the file (a linked library concatenates one offload bundle per
    translation unit in .hip_fatbin)."""
    syms = set()
    with tempfile.TemporaryDirectory() as d:
        fb = Path(d) / "fb.bin"
        subprocess.run([LLVM / "llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, Path(d) / "copy"],
                       check=True, capture_output=True)
        data = fb.read_bytes()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [i for i in range(len(data)) if data.startswith(magic, i)] if magic in data else []
        for n, a in enumerate(starts):
            part, dev = Path(d) / f"b{n}.bin", Path(d) / f"dev{n}.o"
            part.write_bytes(data[a:starts[n + 1] if n + 1 < len(starts) else len(data)])
            r = subprocess.run([LLVM / "clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], capture_output=True)
            if r.returncode != 0:
                continue
            out = subprocess.run([LLVM / "llvm-readelf", "-s", "-W", dev], check=True, capture_output=True,
                                 text=True).stdout
            syms |= {f.split()[-1] for f in out.splitlines() if " FUNC " in f}
    return syms


def host_kernel_handles(lib: Path) -> set:
    """Data objects (weak 'V', or 'd' for kernels with internal linkage) whose demangled name is a function: the kernel
    handles __hipRegisterFunction registers."""
    out = subprocess.run(["nm", "-D", "--defined-only", lib], check=True, capture_output=True, text=True).stdout
    out += subprocess.run(["nm", "--defined-only", lib], capture_output=True, text=True).stdout
    names = {f.split()[-1] for f in out.splitlines() if len(f.split()) == 3 and f.split()[1] in "VvdD"}
    dem = subprocess.run(["c++filt"], input="\n".join(sorted(names)), capture_output=True, text=True).stdout.splitlines()
    return {n for n, d in zip(sorted(names), dem) if d.startswith("void ") and d.endswith(")")}


def main(paths) -> int:
    bad = 0
    for p in map(Path, paths):
        dev, host = device_symbols(p), host_kernel_handles(p)
        missing = sorted(host - dev)
        print(f"{p.name}: {len(host)} kernels registered, {len(dev)} in the gfx950 code object, missing {len(missing)}")
        for m in missing[:10]:
            print("  missing:", m)
        bad |= bool(missing) or not host
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["spmm-research_amd/lib/libspmm_hip.so"]))
