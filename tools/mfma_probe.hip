// tools/mfma_probe.hip -- measurement-only C ABI over spmm_mfma_tile_kernel (round-3/4 measurements: its host
// tables are the round-4 entry layout -- since round 5 the engine permutes each chunk's values, so rebuild this probe only
// against the round-4 header, git show ff75116~1:spmm-research_amd/csrc/spmm_mfma.hpp), driven by
// tools/mfma_probe.py with tile tables from spmm_hip_debug_tiles, before the kernel is wired into the engine.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mfma_probe.hip -o spmm-research_amd/lib/libmfma_probe.so
#include <hip/hip_runtime.h>
#include "../spmm-research_amd/csrc/spmm_kernels.hpp"
#include "../spmm-research_amd/csrc/spmm_mfma.hpp"

using namespace spmm;

extern "C" int mfma_probe_launch(int ntiles, const void *tiles, const void *tchunk, const void *tcolT,
                                 const void *tval, const void *tpos, const void *B, long long b_bytes, void *C,
                                 int ld, int xcd, void *stream) {
    auto st = (hipStream_t)stream;
    if (ntiles <= 0) return 0;
    const int grid = (ntiles + 3) / 4;
    auto t = (const int4 *)tiles;
    auto ch = (const int4 *)tchunk;
    auto tc = (const int32_t *)tcolT;
    auto tv = (const double *)tval;
    auto tp = (const uint16_t *)tpos;
    auto b = (const double *)B;
    auto c = (double *)C;
    if (b_bytes >= (1ll << 32)) return -2;
    if (xcd & 1)
        spmm_mfma_tile_kernel<double, true, 1><<<grid, 256, 0, st>>>(t, ntiles, ch, tc, tv, tp, b, (uint32_t)b_bytes,
                                                                     c, ld);
    else
        spmm_mfma_tile_kernel<double, false, 1><<<grid, 256, 0, st>>>(t, ntiles, ch, tc, tv, tp, b, (uint32_t)b_bytes,
                                                                      c, ld);
    return (int)hipGetLastError();
}
