// tools/mfma_probe_lr.hip -- the experimental low-register tile kernel (tools/mfma_lr.hpp) behind the probe ABI,
// driven by tools/mfma_probe.py --lr-lib.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mfma_probe_lr.hip -o spmm-research_amd/lib/libmfma_probe_lr.so
#include <hip/hip_runtime.h>
#include "../spmm-research_amd/csrc/spmm_kernels.hpp"
#include "mfma_lr.hpp"

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

// variants over all ld columns (a multiple of 32): np 32-column sub-panels per wave, ring B-operand slots
extern "C" int mfma_probe_launch_v(int ntiles, const void *tiles, const void *tchunk, const void *tcolT,
                                   const void *tval, const void *tpos, const void *B, long long b_bytes, void *C,
                                   int ld, int np, int ring, void *stream) {
    auto st = (hipStream_t)stream;
    if (ntiles <= 0) return 0;
    if (b_bytes >= (1ll << 32) || ld % 32) return -2;
    const int grid = (ntiles + 3) / 4;
    auto t = (const int4 *)tiles;
    auto ch = (const int4 *)tchunk;
    auto tc = (const int32_t *)tcolT;
    auto tv = (const double *)tval;
    auto tp = (const uint16_t *)tpos;
    for (int k1 = 0; k1 + 32 <= ld;) {
        const int n = (np == 2 && k1 + 64 <= ld) ? 2 : 1;
        auto b = (const double *)B + k1;
        auto c = (double *)C + k1;
        const uint32_t bb = (uint32_t)(b_bytes - (long long)k1 * 8);
#define GO(NP, R) spmm_mfma_tile_kernel<double, true, NP, R><<<grid, 256, 0, st>>>(t, ntiles, ch, tc, tv, tp, b, bb, c, ld)
        if (n == 2) {
            if (ring == 6) GO(2, 6); else if (ring == 8) GO(2, 8); else GO(2, 12);
        } else {
            if (ring == 6) GO(1, 6); else if (ring == 8) GO(1, 8); else GO(1, 12);
        }
#undef GO
        k1 += 32 * n;
    }
    return (int)hipGetLastError();
}
