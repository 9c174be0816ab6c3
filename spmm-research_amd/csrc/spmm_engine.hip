// spmm_engine.hip -- C ABI (include/spmm_hip.h) of the MI355X-native CSR SpMM engine.
//
// Replaces the reference plugin surface (benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h:9-30):
//   csr_to_format        -> spmm_hip_create + spmm_hip_plan   (validate, copy A to HBM, inspect)
//   Matrix_Format::spmm  -> spmm_hip_run (host x/y, synchronous) / spmm_hip_run_device (HBM-resident)
//   statistics_*         -> spmm_hip_stats_labels / spmm_hip_stats
// Device kernels: spmm_kernels.hpp.
//
// The inspector (plan, per K; untimed like the reference's csr_to_format) decides the work shape from the matrix:
//   * row group width G and lane width VEC from the K-panel width (16-byte lanes where the layout allows);
//   * block capacity cap: 2048 nonzeros (the LDS capacity), smaller for small matrices so at least ~1024 blocks
//     (4 per CU) exist;
//   * split length T (split_length(): 64..2048 from a time model of the launch): rows longer than T become
//     ceil(len/T) virtual rows so no serial chain of memory round trips outlasts the rest of the grid; blocks
//     holding long rows are dispatched first.  Rows of <= T nonzeros are summed exactly like the reference
//     (bit-identical); split rows are combined in slot order (deterministic).  SPMM_HIP_SEQ_MAX=<n> overrides T
//     (n >= 2048 keeps every row <= 2048 bit-exact);
//   * K panels: when B (ncols*K*s) would crowd the Infinity Cache (> 128 MB) and the gather dominates (>= 16
//     nonzeros per row), K is cut into panels of 256-byte B rows (32 fp64 / 64 fp32 columns; SPMM_HIP_PANEL_K=<cols>
//     overrides), one launch per panel (A is re-streamed per panel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/spmm_hip.h"
#include "spmm_handle.hpp"
#include "spmm_kernels.hpp"
#include "spmm_mfma.hpp"

using namespace spmm;
using namespace spmm_engine;

namespace spmm_engine {
thread_local std::string g_detail;
int fail(int status, const std::string &what) {
    g_detail = what;
    return status;
}
}  // namespace spmm_engine

namespace {

#define HIPCHK(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess)                                                                            \
            return fail(_e == hipErrorOutOfMemory ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP,                \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                              \
    } while (0)

constexpr int CAP = 2048;         // LDS capacity of a block (nonzeros)
constexpr int CAP_BIG = 4096;     // the wide window: SPMM_HIP_CAP=4096, 16-byte lanes, groups of >= 8 lanes
constexpr int64_t WIDE_MIN_NNZ = 2500000;   // policy: the wide window for fp64 matrices this large ...
constexpr double WIDE_MIN_ROW = 256.0;      // ... whose rows average this many nonzeros (§6.43)
constexpr int PAD_BYTES = 64;     // device col/val padding (16-byte staging may read up to 3 elements past nnz)
// LDS B tiles (spmm_tile_kernel)
#ifndef SPMM_TILE_UCB_KB
#define SPMM_TILE_UCB_KB 12                // A/B builds only
#endif
#ifndef SPMM_TILE_CAPA
#define SPMM_TILE_CAPA 896
#endif
constexpr int TILE_UCB = SPMM_TILE_UCB_KB * 1024;   // LDS bytes of staged B rows per chunk (two chunk buffers per workgroup)
constexpr int TILE_CAPA = SPMM_TILE_CAPA;           // entries per chunk (LDS; a multiple of 8; 3 workgroups per CU incl. 512-B granules)
constexpr int TILE_WIDE_DEFAULT = 1;      // SPMM_HIP_TILE_WIDE: tile compute-lane width, 16-byte pieces
constexpr int TILE_RMAX = 64;             // rows per tile (row groups x rows per group)
constexpr int64_t TILE_POLICY_MAX_ROW = 256;   // policy: staged B rows of at most 256 B (K=64 fp64 lost 6-26 %, §6.9)
constexpr int TILE_MIN_BUILT = 64;         // policy: fewer built tiles than this run as one serial tail (§6.9)
constexpr double TILE_MIN_REUSE = 8.0;    // policy: sampled reuse (nnz per union column) to leave the row kernel (§6.9)
constexpr int64_t TILE_MIN_TILES = 512;   // policy: candidate tiles (one workgroup each) to fill 256 CUs twice (§6.9:
                                          // 76-173 tiles ran 2.7-3x slower than the row kernel's split rows)
                                          // (measured, DESIGN §6.9: 1.22x at ~14 on 39 K x 500 bw 0.05; 0.66-0.82x
                                          // at 4.5-6; the kernel is LDS-throughput bound)
constexpr int TILE_ROWS = 32;             // rows per tile (32: 1.22x vs 64: 1.19x on the dense band; more tiles)
constexpr int TILE_SEG_ALIGN = 4;         // row segments padded to this many entries (value -0, the zero B row)
constexpr uint16_t TILE_PAD_LIDX = 0xFFFF;   // chunk-local column of a padding entry
// Matrix-core tiles (spmm_mfma_tile_kernel): fp64 and fp32, K a multiple of 32, rows with strictly
// increasing columns, B below 4 GiB (32-bit buffer offsets).  Policy (the cost-model gate, mfma_sample / mfma_cost,
// DESIGN §6.18): 16-row tiles with enough nonzeros per chunk, taken when the model's time beats the row kernel's.
constexpr double MFMA_TILE_REUSE = 2.0;     // per tile: reuse (nonzeros per union column) floor, and MFMA_TILE_NPC
// Leftover rows of a plan whose tiles hold more than 1 - GAP_SHORT_FRAC of the nonzeros run as pieces of at most
// GAP_SEQ_MAX nonzeros (a lone long row would otherwise be a serial straggler after the tile kernel).
constexpr double GAP_SHORT_FRAC = 0.125;
constexpr int GAP_SEQ_MAX = 64;

int pow2_ceil(int64_t x) {
    int p = 1;
    while (p < x && p < (1 << 30)) p <<= 1;
    return p;
}


int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// Lane layout for a panel of `kw` columns with row stride `ld`: VEC values per lane (16-byte lanes when every lane
// address stays 16-byte aligned), G lanes per row group (power of two, <= 64).
void lane_layout(int kw, int ld, size_t vsize, int &vec, int &g) {
    const size_t lb = (size_t)ld * vsize, wb = (size_t)kw * vsize;
    if (lb % 16 == 0 && wb % 16 == 0)
        vec = (int)(16 / vsize);
    else if (lb % 8 == 0 && wb % 8 == 0 && vsize <= 8)
        vec = (int)(8 / vsize);
    else
        vec = 1;
    g = std::min(64, pow2_ceil(std::max(1, (kw + vec - 1) / vec)));
}

void free_plan(spmm_hip_t *h) {
    void *ps[] = {h->d_b, h->d_xcol, h->d_c, h->d_part, h->d_vrow_ptr, h->d_vdest, h->d_blk, h->d_long_rows,
                  h->d_wcol, h->d_wval, h->d_lr_cnt, h->d_slot_lr, h->d_tiles, h->d_tchunk, h->d_tcol, h->d_tseg,
                  h->d_tlidx, h->d_tval, h->d_tstamps, h->d_wperm, h->d_tperm, h->d_mflag};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    h->d_b = h->d_xcol = h->d_c = h->d_part = nullptr;
    h->d_wcol = nullptr;
    h->d_wval = nullptr;
    h->d_lr_cnt = h->d_slot_lr = nullptr;
    h->d_tiles = h->d_tchunk = nullptr;
    h->d_tcol = nullptr;
    h->d_tseg = h->d_tlidx = nullptr;
    h->d_tval = nullptr;
    h->d_tstamps = nullptr;
    h->d_wperm = h->d_tperm = nullptr;
    h->d_mflag = nullptr;
    h->nwperm = h->ntperm = 0;
    h->fuse = false;
    h->win_blk.clear();
    h->win_v.clear();
    h->d_vrow_ptr = h->d_vdest = nullptr;
    h->d_blk = nullptr;
    h->d_long_rows = nullptr;
    h->b_bytes = h->c_bytes = h->insp_bytes = 0;
    h->plan = Plan();
    h->nv = h->nblk = h->nlong = h->nslots = 0;
    h->last_x = nullptr;
}

// ---------------------------------------------------------------------------------------------------- launches
template <typename T, int VEC, int G, int U, bool NTC, bool DMA, bool BUF>
void launch_rows_v(spmm_hip_t *h, const T *B, T *C, T *P, int ld, int kw, hipStream_t s) {
    const uint32_t bb = (uint32_t)std::min<uint64_t>((uint64_t)h->ncols * ld * sizeof(T), 0xFFFFFFFFull);
    if (h->plan.nwin > 1) {
        // chained mode: one launch per column window, in window order (each continues the chains of the last)
        const int lmax = h->plan.lmax;
        auto gow = [&](auto vl_c) {
            for (int w = 0; w < h->plan.nwin; ++w) {
                const int b0 = h->win_blk[w], nb = h->win_blk[w + 1] - b0;
                if (nb == 0) continue;
                spmm_rows_kernel<T, VEC, G, U, CAP, NTC, DMA, BUF, DEST_CHAIN, false, decltype(vl_c)::value>
                    <<<nb, WG, 0, s>>>(h->d_vrow_ptr, h->d_wcol, (const T *)h->d_wval, h->d_blk + b0, nb, h->d_vdest,
                                       B, C, P, ld, kw, bb, lmax, nullptr, nullptr, nullptr, 0u);
            }
        };
        if (lmax > 1) gow(std::true_type()); else gow(std::false_type());
        return;
    }
    // partial slots of this panel as one buffer resource (the fused path needs them below 4 GiB; checked at plan)
    const uint32_t pb = (uint32_t)std::min<uint64_t>((uint64_t)h->nslots * ld * sizeof(T), 0xFFFFFFFFull);
    auto go = [&](auto mode_c, auto xcd_c, auto vl_c, auto pair_c) {
        auto run = [&](auto cap_c) {
            spmm_rows_kernel<T, VEC, G, U, decltype(cap_c)::value, NTC, DMA, BUF, decltype(mode_c)::value,
                             decltype(xcd_c)::value, decltype(vl_c)::value, decltype(pair_c)::value>
                <<<dim3(h->nblk, h->plan.ygrid ? h->plan.npanels : 1), WG, 0, s>>>(
                h->d_vrow_ptr, h->d_col, (const T *)h->d_val, h->d_blk, h->nblk, h->d_vdest, B, C, P, ld, kw, bb,
                h->plan.lmax, h->fuse ? h->d_lr_cnt : nullptr, h->d_slot_lr, h->d_long_rows, pb);
        };
        // the wide window (blocks of up to CAP_BIG nonzeros): 16-byte lanes, groups of >= 8 lanes, no pairing
        if constexpr (VEC * sizeof(T) == 16 && G >= 8 && !decltype(pair_c)::value && U > 0) {
            if (h->plan.cap > CAP) {
                run(std::integral_constant<int, CAP_BIG>());
                return;
            }
        }
        run(std::integral_constant<int, CAP>());
    };
    using split_c = std::integral_constant<int, DEST_SPLIT>;
    using row_c = std::integral_constant<int, DEST_ROW>;
    using T_ = std::true_type;
    using F_ = std::false_type;
    const bool vl = h->plan.lmax > 1, sp = h->d_vdest != nullptr;   // split rows, or rows left to tiles
    if constexpr (U > 1 && G > 1) {
        if (h->plan.pair) {              // paired short rows
            if (h->plan.xcd) {
                if (sp) vl ? go(split_c(), T_(), T_(), T_()) : go(split_c(), T_(), F_(), T_());
                else vl ? go(row_c(), T_(), T_(), T_()) : go(row_c(), T_(), F_(), T_());
            } else {
                if (sp) vl ? go(split_c(), F_(), T_(), T_()) : go(split_c(), F_(), F_(), T_());
                else vl ? go(row_c(), F_(), T_(), T_()) : go(row_c(), F_(), F_(), T_());
            }
            return;
        }
    }
    if (h->plan.xcd) {
        if (sp) vl ? go(split_c(), T_(), T_(), F_()) : go(split_c(), T_(), F_(), F_());
        else vl ? go(row_c(), T_(), T_(), F_()) : go(row_c(), T_(), F_(), F_());
    } else {
        if (sp) vl ? go(split_c(), F_(), T_(), F_()) : go(split_c(), F_(), F_(), F_());
        else vl ? go(row_c(), F_(), T_(), F_()) : go(row_c(), F_(), F_(), F_());
    }
}

// 32-bit buffer offsets for the B gather are valid while B fits 4 GiB.
inline bool buf_ok(const spmm_hip_t *h, int ld) { return (uint64_t)h->ncols * (uint64_t)ld * h->vsize < (1ULL << 32); }

#ifdef SPMM_TUNING
// Tuning build only: a grid of row-kernel variants for the fp64 16-byte-lane shapes, selected at run time.
template <typename T, int VEC, int G, int U, bool NTC, bool DMA, bool BUF>
bool try_variant(spmm_hip_t *h, const T *B, T *C, T *P, int ld, int kw, hipStream_t s) {
    const Variant &v = h->var;
    if (v.u != U || v.ntc != (int)NTC || v.dma != (int)DMA || v.buf != (int)BUF) return false;
    launch_rows_v<T, VEC, G, U, NTC, DMA, BUF>(h, B, C, P, ld, kw, s);
    return true;
}
#define TV(U, NTC, DMA, BUF) try_variant<T, VEC, G, U, NTC, DMA, BUF>(h, B, C, P, ld, kw, s) ||
template <typename T, int VEC, int G>
bool launch_tuned(spmm_hip_t *h, const T *B, T *C, T *P, int ld, int kw, hipStream_t s) {
    return TV(16, true, true, false) TV(16, true, false, false) TV(16, true, true, true) TV(16, true, false, true)
        TV(-8, true, false, true) TV(-16, true, false, true) false;
}
#endif

template <typename T, int VEC, int G>
void launch_rows_t(spmm_hip_t *h, const T *B, T *C, T *P, int ld, int kw, hipStream_t s) {
#ifdef SPMM_TUNING
    if constexpr (std::is_same<T, double>::value && ((VEC == 2 && G >= 4 && G <= 32) || (VEC == 1 && G == 1))) {
        if (launch_tuned<T, VEC, G>(h, B, C, P, ld, kw, s)) return;
    }
#endif
    // One-lane row groups (K = 1): LDS-DMA staging and flat gathers (0.086 vs 0.121 ms on config 2, K=1); wider
    // groups: staging through VGPRs and 32-bit buffer-offset gathers (config 2 K=32 0.404 vs 0.420 ms; 500-nnz rows
    // K=8 2.10 vs 2.91 ms) -- DESIGN.md §6.2.
    constexpr bool dma = G == 1 ? true : (bool)DEF_DMA;
    constexpr bool buf = G == 1 ? false : (bool)DEF_BUF;
    if (buf && !buf_ok(h, ld))
        launch_rows_v<T, VEC, G, DEF_U, (bool)DEF_NTC, dma, false>(h, B, C, P, ld, kw, s);
    else
        launch_rows_v<T, VEC, G, DEF_U, (bool)DEF_NTC, dma, buf>(h, B, C, P, ld, kw, s);
}

template <typename T, int VEC>
void launch_rows_g(spmm_hip_t *h, int g, const T *B, T *C, T *P, int ld, int kw, hipStream_t s) {
    switch (g) {
        case 1: launch_rows_t<T, VEC, 1>(h, B, C, P, ld, kw, s); break;
        case 2: launch_rows_t<T, VEC, 2>(h, B, C, P, ld, kw, s); break;
        case 4: launch_rows_t<T, VEC, 4>(h, B, C, P, ld, kw, s); break;
        case 8: launch_rows_t<T, VEC, 8>(h, B, C, P, ld, kw, s); break;
        case 16: launch_rows_t<T, VEC, 16>(h, B, C, P, ld, kw, s); break;
        case 32: launch_rows_t<T, VEC, 32>(h, B, C, P, ld, kw, s); break;
        default: launch_rows_t<T, VEC, 64>(h, B, C, P, ld, kw, s); break;
    }
}

template <typename T>
void launch_panel(spmm_hip_t *h, const T *B, T *C, T *P, int ld, int kw, hipStream_t s) {
    int vec, g;
    lane_layout(kw, ld, sizeof(T), vec, g);
    if (vec == 16 / (int)sizeof(T)) {
        if constexpr (sizeof(T) == 8)
            launch_rows_g<T, 2>(h, g, B, C, P, ld, kw, s);
        else
            launch_rows_g<T, 4>(h, g, B, C, P, ld, kw, s);
    } else if (vec == 2 && sizeof(T) == 4) {
        launch_rows_g<T, 2>(h, g, B, C, P, ld, kw, s);
    } else {
        launch_rows_g<T, 1>(h, g, B, C, P, ld, kw, s);
    }
}

// Tile kernel for a panel: 16-byte lanes (checked at plan), G lanes per row group, tile_rpg(G) rows per group.
template <typename T, int G>
void launch_tiles_g(spmm_hip_t *h, const T *B, T *C, int ld, int kw, hipStream_t s) {
    constexpr int VEC = 16 / (int)sizeof(T);
    constexpr int NG = WG / G;
    constexpr int RPG = NG * 8 <= TILE_RMAX ? 8 : (TILE_RMAX / NG > 1 ? TILE_RMAX / NG : 1);
    auto go = [&](auto xcd_c, auto s_c) {
        constexpr int SW = decltype(s_c)::value;
        spmm_tile_kernel<T, VEC, G, RPG / SW, TILE_UCB, TILE_CAPA, (bool)DEF_NTC, decltype(xcd_c)::value, SW>
            <<<h->plan.ntile, WG, 0, s>>>(h->d_tiles, h->d_tchunk, h->d_tcol, h->d_tseg, (const T *)h->d_tval,
                                           h->d_tlidx, B, C, ld, h->d_tstamps);
    };
    // S = 4 measured 1.3-2x slower everywhere and is not instantiated; S = 2 stays selectable
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, (RPG % 2 == 0 && G >= 2) ? 2 : 1>;
    auto go_x = [&](auto s_c) {
        if (h->plan.tile_xcd) go(std::true_type(), s_c); else go(std::false_type(), s_c);
    };
    if (h->plan.tile_wide == 2) go_x(S2());
    else go_x(S1());
}

template <typename T>
void launch_tiles(spmm_hip_t *h, const T *B, T *C, int ld, int kw, hipStream_t s) {
    int vec, g;
    lane_layout(kw, ld, sizeof(T), vec, g);
    switch (g) {
        case 4: launch_tiles_g<T, 4>(h, B, C, ld, kw, s); break;     // (B rows >= 64 bytes: G >= 4, checked at plan)
        case 8: launch_tiles_g<T, 8>(h, B, C, ld, kw, s); break;
        case 16: launch_tiles_g<T, 16>(h, B, C, ld, kw, s); break;
        case 32: launch_tiles_g<T, 32>(h, B, C, ld, kw, s); break;
        default: launch_tiles_g<T, 64>(h, B, C, ld, kw, s); break;
    }
}

// Matrix-core tiles over all K columns (a multiple of 32): four 16-row tiles (one per wave) per workgroup; a wave owns
// 64 columns (two 32-column sub-panels, NP = 2) where two are left, else 32 (SPMM_HIP_MFMA_NP=1 keeps
// 32).  The buffer descriptor of B covers the rest of the array from the sub-panel on.
// B-operand ring (spmm_mfma.hpp): 0 = per sub-panel count default, else SPMM_HIP_MFMA_RING = 6 or 12 slots
constexpr int MFMA_RING_NP1 = 6, MFMA_RING_NP2 = 6;   // r05b: 6 slots 0.94-1.03x at 32 columns, 0.87-1.02x at 64
template <typename T>
void launch_mfma(spmm_hip_t *h, const T *B, T *C, int K, hipStream_t s) {
    const int grid = (h->plan.ntile + 3) / 4;
    const int np_max = env_int("SPMM_HIP_MFMA_NP", 2) >= 2 ? 2 : 1;
    const int ring_env = env_int("SPMM_HIP_MFMA_RING", 0);
    for (int k1 = 0; k1 + 32 <= K;) {
        const int np = (np_max >= 2 && k1 + 64 <= K) ? 2 : 1;
        const int ring = ring_env == 6 || ring_env == 12 ? ring_env : np == 2 ? MFMA_RING_NP2 : MFMA_RING_NP1;
        const uint32_t bb = (uint32_t)(((size_t)h->ncols * (size_t)K - (size_t)k1) * sizeof(T));
        auto go = [&](auto xcd_c, auto np_c, auto r_c) {
            spmm_mfma_tile_kernel<T, decltype(xcd_c)::value, decltype(np_c)::value, decltype(r_c)::value>
                <<<grid, WG, 0, s>>>(h->d_tiles, h->plan.ntile, h->d_tchunk, h->d_tcol, (const T *)h->d_tval,
                                     h->d_tlidx, B + k1, bb, C + k1, K);
        };
        using N1 = std::integral_constant<int, 1>;
        using N2 = std::integral_constant<int, 2>;
        using R6 = std::integral_constant<int, 6>;
        using R12 = std::integral_constant<int, MFMA_KS>;
        auto go_r = [&](auto xcd_c) {
            if (np == 2) ring == 6 ? go(xcd_c, N2(), R6()) : go(xcd_c, N2(), R12());
            else ring == 6 ? go(xcd_c, N1(), R6()) : go(xcd_c, N1(), R12());
        };
        if (h->plan.tile_xcd) go_r(std::true_type());
        else go_r(std::false_type());
        k1 += 32 * np;
    }
}

// The matrix-core tiles' exact range (spmm_mfma.hpp): B's check, on the row kernel's stream (beside the tiles when
// that is the side stream) -- an out-of-range B stores this launch's sequence number into mflag[1] (no reset launch;
// under a graph replay a baked-in number can only keep the exact fallback on, never skip it).  One slot per handle:
// this relies on the handle's contract that its runs are serialised on one stream (include/spmm_hip.h,
// spmm_hip_run_device) -- a later launch's flag can then only be stored after this launch's fix-up has read it ...
template <typename T>
int launch_mfma_check(spmm_hip_t *h, const T *B, int K, hipStream_t rs) {
    h->mflag_seq = h->mflag_seq == INT32_MAX ? 1 : h->mflag_seq + 1;
    const int64_t n = (int64_t)h->ncols * K;
    const int64_t nv = (n + 16 / (int64_t)sizeof(T) - 1) / (16 / (int64_t)sizeof(T));
    const unsigned rg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, (nv + WG - 1) / WG));
    mfma_range_kernel<T><<<rg, WG, 0, rs>>>(B, n, h->d_mflag + 1, h->mflag_seq);
    return h->mflag_seq;
}

// ... and after the tiles and the check (the join): every tile recomputed by the sparse IEEE chain when A or B is out
// of range, else an immediate exit
template <typename T>
void launch_mfma_fixup(spmm_hip_t *h, const T *B, T *C, int K, int seq, hipStream_t s) {
    const int grid = std::min((h->plan.ntile + 3) / 4, 512);
    mfma_fixup_kernel<T><<<grid, WG, 0, s>>>(h->d_tiles, h->plan.ntile, h->d_tchunk, h->d_tcol, (const T *)h->d_tval,
                                             h->d_tlidx, B, C, K, K, h->d_mflag, seq);
}

// rs: the stream of the row kernel and the combine (the launch stream, or the handle's side stream when the row kernel
// only runs the leftover rows of a matrix-core plan, concurrently with the tiles on s)
template <typename T>
void launch_spmm_t(spmm_hip_t *h, const T *B, T *C, int K, hipStream_t s, hipStream_t rs, int *seq) {
    T *P = (T *)h->d_part;
    const bool mf = h->plan.ntile > 0 && h->plan.tile_mfma;
    if (mf) *seq = launch_mfma_check<T>(h, B, K, rs);
    // matrix-core tiles: one pass over all K columns (the row kernel's K panels are for its B gather, not theirs)
    if (mf) launch_mfma<T>(h, B, C, K, s);
    for (int p = 0; p < h->plan.npanels; ++p) {
        const int k0 = p * h->plan.kw;
        const int kw = std::min(h->plan.kw, K - k0);
        // ygrid: every panel of the row kernel in one launch (blockIdx.y = panel; equal panel widths, checked at plan)
        if (h->nblk > 0 && (!h->plan.ygrid || p == 0)) launch_panel<T>(h, B + k0, C + k0, P ? P + k0 : nullptr, K, kw, rs);
        if (h->plan.ntile > 0 && !h->plan.tile_mfma) launch_tiles<T>(h, B + k0, C + k0, K, kw, s);
    }
    if (h->nlong > 0 && !h->fuse) {
        spmm_combine_kernel<T><<<h->nlong, WG, 0, rs>>>(h->d_long_rows, P, C, K);
    }
}

int launch_spmm(spmm_hip_t *h, const void *B, void *C, int K, hipStream_t s) {
    // matrix-core plans: the exact-range check of B and the leftover rows (a skewed row's pieces, low-reuse tiles) run
    // beside the tile kernel; the fix-up follows the join
    const bool mf = h->plan.tile_mfma && h->plan.ntile > 0;
    const bool par = mf && h->side;
    if (par) {
        HIPCHK(hipEventRecord(h->ev_fork, s));
        HIPCHK(hipStreamWaitEvent(h->side, h->ev_fork, 0));
    }
    hipStream_t rs = par ? h->side : s;
    int seq = 0;
    const bool f64 = h->dtype == SPMM_HIP_F64;
    if (f64)
        launch_spmm_t<double>(h, (const double *)B, (double *)C, K, s, rs, &seq);
    else
        launch_spmm_t<float>(h, (const float *)B, (float *)C, K, s, rs, &seq);
    if (par) {
        HIPCHK(hipEventRecord(h->ev_join, h->side));
        HIPCHK(hipStreamWaitEvent(s, h->ev_join, 0));
    }
    if (mf) {
        if (f64) launch_mfma_fixup<double>(h, (const double *)B, (double *)C, K, seq, s);
        else launch_mfma_fixup<float>(h, (const float *)B, (float *)C, K, seq, s);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SPMM_HIP_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return SPMM_HIP_OK;
}

}  // namespace

namespace spmm_engine {
// The handle's own row-major B, column-major staging and C buffers for the planned k, allocated at first use (host
// runs, column-major device input, spmm_hip_device_ptrs, multi-GPU shards) -- not at plan time.
int ensure_buffers(spmm_hip_t *h, bool b, bool xcol, bool c) {
    HIPCHK(hipSetDevice(h->device));
    if (b && !h->d_b) HIPCHK(hipMalloc(&h->d_b, h->b_bytes));
    if (xcol && !h->d_xcol) HIPCHK(hipMalloc(&h->d_xcol, h->b_bytes));
    if (c && !h->d_c) HIPCHK(hipMalloc(&h->d_c, h->c_bytes));
    return SPMM_HIP_OK;
}

int launch_transpose(spmm_hip_t *h, const void *X, void *Bt, int K, hipStream_t s) {
    if (h->ncols == 0 || K == 0) return SPMM_HIP_OK;
    dim3 grid((unsigned)((h->ncols + 63) / 64), (unsigned)((K + 31) / 32));
    if (h->dtype == SPMM_HIP_F64)
        transpose_colmajor_kernel<double><<<grid, WG, 0, s>>>((const double *)X, (double *)Bt, h->ncols, K);
    else
        transpose_colmajor_kernel<float><<<grid, WG, 0, s>>>((const float *)X, (float *)Bt, h->ncols, K);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SPMM_HIP_ERR_HIP, std::string("transpose launch: ") + hipGetErrorString(e));
    return SPMM_HIP_OK;
}
}  // namespace spmm_engine

namespace {

// ------------------------------------------------------------------------------------------------- inspector
// Split length T.  A row is one serial chain of len/U dependent gather batches; measured on MI355X (§6.2) a chain
// advances ~5.5 nonzeros/us under load, and a launch takes about est' = 1.3 * (gathered B rows at ~12 TB/s incl.
// L2 hits + A and C streamed at ~6 TB/s) + 10 us.  Rows whose chain would outlast the launch are split (their
// blocks are dispatched first, see inspect()); rows within 2.5x of the mean are never split (splitting them
// balances nothing and adds partial-sum traffic), unless the matrix has too few rows to give every CU work
// (m < 2048), where every row is cut so the row groups of a block have work.  T is clamped to [64, 2048].
// Rows <= T stay a single FMA chain, bit-identical to the reference; config 2 (T = 2048) is exact throughout.
constexpr double CHAIN_NNZ_PER_US = 5.5;
int split_length(const spmm_hip_t *h, int kw) {
    const double s = (double)h->vsize;
    const double est_us = 1.3 * ((double)h->nnz * kw * s / 12.0e6 +
                                 ((double)h->nnz * (4.0 + s) + (double)h->m * kw * s + 4.0 * h->m) / 6.0e6) + 10.0;
    double t = CHAIN_NNZ_PER_US * est_us * (double)h->var.u / 16.0;
    // rows at least 2.5x the mean stay whole: splitting every row of a small long-row matrix (698 x 500) is 1.4-4.7x
    // slower than whole rows with vector lanes (profiles/r02_small_split.jsonl)
    const double mean = (double)h->nnz / (double)std::max<int64_t>(h->m, 1);
    if (h->m >= 2048 || mean >= 32.0) t = std::max(t, 2.5 * mean);
    return (int)std::max(64.0, std::min((double)CAP, t));
}

constexpr int64_t PANEL_ROW_BYTES = 256;          // B bytes per row of one K panel
constexpr int64_t SMALL_NNZ = 1000000;            // small-matrix panels (ygrid) below this many nonzeros
#ifndef SMALL_KW_DEFAULT
#define SMALL_KW_DEFAULT 0
#endif
constexpr double PANEL_MIN_B_BYTES = 128.0 * (1 << 20);  // B below half the Infinity Cache: no panels
constexpr double PANEL_MIN_ROW_NNZ = 16.0;

struct Inspection {
    std::vector<int32_t> vrow_ptr, vdest;
    std::vector<int2> blk;
    std::vector<int4> long_rows;
    std::vector<int> win_blk;       // chained mode: block offsets per window
    std::vector<int64_t> win_v;     // chained mode: virtual-row offsets per window
    std::vector<int64_t> perm;      // chained mode: position in the window-major arrays -> original nonzero
    int heavy = 0;  // blocks moved to the front of the table
    int nslots = 0;
    int64_t ngaps = 0;  // gap virtual rows (runs of rows computed by the tile kernel, never in a block)
};

// Pack virtual rows [v0, v1) greedily into blocks of <= cap nonzeros and <= CAP_ROWS virtual rows, appended to out.
// Longest-first for blocks whose longest row is a long serial chain (>= 256 nonzeros and >= 8x the mean row):
// they are dispatched first and overlap the rest of the grid.  Everything else keeps row order, so all XCDs
// sweep the same B window together.
void pack_blocks(const std::vector<int32_t> &vp, int64_t v0, int64_t v1, int cap, Inspection &out,
                 bool heavy_first = true, int max_rows = CAP_ROWS) {
    std::vector<int2> order;
    std::vector<int32_t> longest;
    int64_t start = v0;
    int32_t lmax = 0;
    for (int64_t v = v0; v <= v1; ++v) {
        const int64_t len = v < v1 ? (int64_t)vp[v + 1] - vp[v] : 0;
        if (v == v1 || (v > start && (v - start >= max_rows || (int64_t)vp[v] - vp[start] + len > cap))) {
            if (v > start) {
                order.push_back(make_int2((int)start, (int)v));
                longest.push_back(lmax);
            }
            start = v;
            lmax = 0;
        }
        lmax = std::max<int32_t>(lmax, (int32_t)len);
    }
    const double mean = v1 > v0 ? (double)(vp[v1] - vp[v0]) / (double)(v1 - v0) : 0.0;
    const int32_t heavy_len = heavy_first ? (int32_t)std::max(256.0, 8.0 * mean) : INT32_MAX;
    std::vector<int> hv;
    for (size_t b = 0; b < order.size(); ++b)
        if (longest[b] >= heavy_len) hv.push_back((int)b);
    std::stable_sort(hv.begin(), hv.end(), [&](int a, int b) { return longest[a] > longest[b]; });
    out.heavy += (int)hv.size();
    for (int b : hv) out.blk.push_back(order[b]);
    for (size_t b = 0; b < order.size(); ++b)
        if (longest[b] < heavy_len) out.blk.push_back(order[b]);
}

// Virtual rows (rows longer than T cut into T-nonzero pieces) packed into blocks (one column window).
// skip (optional): rows computed elsewhere (tiles).  A run of skipped rows becomes one GAP virtual row (destination
// 0, never in a block) so the virtual-row offsets stay one prefix array; blocks never cross a gap.
// piece: length of the pieces rows longer than T are cut into (0 = T).
void inspect(const int32_t *rp, int64_t m, int T, int cap, Inspection &out, bool heavy_first = true,
             const uint8_t *skip = nullptr, int max_rows = CAP_ROWS, int piece = 0) {
    const int P = piece > 0 ? piece : T;
    out = Inspection();
    out.vrow_ptr.reserve((size_t)m + 1);
    out.vrow_ptr.push_back(rp[0]);
    bool any_split = false;
    std::vector<int64_t> gaps;     // virtual-row index of each gap
    for (int64_t r = 0; r < m; ++r) {
        const int64_t len = (int64_t)rp[r + 1] - rp[r];
        if (skip && skip[r]) {
            int64_t r1 = r;
            while (r1 < m && skip[r1]) ++r1;
            gaps.push_back((int64_t)out.vrow_ptr.size() - 1);
            out.vrow_ptr.push_back(rp[r1]);
            out.vdest.push_back(0);
            r = r1 - 1;
            continue;
        }
        if (len <= T) {
            out.vrow_ptr.push_back(rp[r + 1]);
            out.vdest.push_back((int32_t)r);
        } else {
            any_split = true;
            const int pieces = (int)((len + P - 1) / P);
            out.long_rows.push_back(make_int4((int)r, out.nslots, pieces, 0));
            for (int q = 0; q < pieces; ++q) {
                out.vrow_ptr.push_back((int32_t)std::min<int64_t>((int64_t)rp[r] + (int64_t)(q + 1) * P, rp[r + 1]));
                out.vdest.push_back(-(out.nslots + q) - 1);
            }
            out.nslots += pieces;
        }
    }
    if (!any_split && gaps.empty()) out.vdest.clear();
    out.ngaps = (int64_t)gaps.size();
    const int64_t nv = (int64_t)out.vrow_ptr.size() - 1;
    int64_t v0 = 0;
    for (int64_t gv : gaps) {
        if (gv > v0) pack_blocks(out.vrow_ptr, v0, gv, cap, out, heavy_first, max_rows);
        v0 = gv + 1;
    }
    if (nv > v0) pack_blocks(out.vrow_ptr, v0, nv, cap, out, heavy_first, max_rows);
}

// Every row's columns non-decreasing (coo_to_csr's output).  Column windows keep each row's CSR order only then.
bool rows_sorted(const int32_t *rp, const int32_t *col, int64_t m) {
    for (int64_t r = 0; r < m; ++r)
        for (int64_t j = (int64_t)rp[r] + 1; j < rp[r + 1]; ++j)
            if (col[j] < col[j - 1]) return false;
    return true;
}
// every row's columns strictly increasing (no repeated column: one panel cell per entry)
bool rows_strict(const int32_t *rp, const int32_t *col, int64_t m) {
    for (int64_t r = 0; r < m; ++r)
        for (int64_t j = (int64_t)rp[r] + 1; j < rp[r + 1]; ++j)
            if (col[j] <= col[j - 1]) return false;
    return true;
}

// Pieces of the row split (rows <= T whole, longer rows in T-nonzero pieces to partial slots), in row order:
// {destination (C row >= 0, slot -s-1), first nonzero, end}.
struct Piece {
    int32_t d;
    int32_t s, e;
};
void make_pieces(const int32_t *rp, int64_t m, int T, std::vector<Piece> &pcs, Inspection &out) {
    pcs.clear();
    pcs.reserve((size_t)m);
    for (int64_t r = 0; r < m; ++r) {
        const int64_t len = (int64_t)rp[r + 1] - rp[r];
        if (len <= T) {
            pcs.push_back({(int32_t)r, rp[r], rp[r + 1]});
        } else {
            const int pieces = (int)((len + T - 1) / T);
            out.long_rows.push_back(make_int4((int)r, out.nslots, pieces, 0));
            for (int q = 0; q < pieces; ++q)
                pcs.push_back({-(out.nslots + q) - 1, (int32_t)(rp[r] + (int64_t)q * T),
                               (int32_t)std::min<int64_t>((int64_t)rp[r] + (int64_t)(q + 1) * T, rp[r + 1])});
            out.nslots += pieces;
        }
    }
}

// Segments a piece would make with windows of W columns (the window index changes along the sorted row).
int64_t count_segments(const std::vector<Piece> &pcs, const int32_t *col, int64_t W) {
    int64_t n = 0;
    for (const Piece &p : pcs) {
        if (p.s == p.e) {
            ++n;
            continue;
        }
        int64_t last = -1;
        for (int32_t j = p.s; j < p.e; ++j) {
            const int64_t w = col[j] / W;
            n += (w != last);
            last = w;
        }
    }
    return n;
}

// Chained mode (column windows of W columns): every piece is cut where its column window changes; window w's
// segments form the virtual rows of launch w, in row order, their nonzeros copied window-major (perm).  A
// segment's vdest is (d << 1) | cont, cont = 1 unless it is the piece's first segment (the chain continues from
// the value the previous window stored).  Empty rows get one empty segment in window 0 (they store 0).
void inspect_windows(const int32_t *rp, const int32_t *col, int64_t m, int64_t ncols, int T, int cap, int64_t W,
                     Inspection &out, int max_rows = CAP_ROWS) {
    out = Inspection();
    std::vector<Piece> pcs;
    make_pieces(rp, m, T, pcs, out);
    const int nwin = (int)((ncols + W - 1) / W);
    std::vector<int64_t> nseg_w(nwin + 1, 0), nnz_w(nwin + 1, 0);
    for (const Piece &p : pcs) {
        if (p.s == p.e) {
            ++nseg_w[0];
            continue;
        }
        int64_t last = -1;
        for (int32_t j = p.s; j < p.e; ++j) {
            const int64_t w = col[j] / W;
            nseg_w[w] += (w != last);
            ++nnz_w[w];
            last = w;
        }
    }
    std::vector<int64_t> seg_off(nwin + 1, 0), nz_off(nwin + 1, 0);
    for (int w = 0; w < nwin; ++w) {
        seg_off[w + 1] = seg_off[w] + nseg_w[w];
        nz_off[w + 1] = nz_off[w] + nnz_w[w];
    }
    const int64_t nseg = seg_off[nwin];
    out.vrow_ptr.assign((size_t)nseg + 1, 0);
    out.vdest.assign((size_t)nseg, 0);
    out.perm.assign((size_t)nz_off[nwin], 0);
    std::vector<int64_t> sc(seg_off.begin(), seg_off.end() - 1), nc(nz_off.begin(), nz_off.end() - 1);
    for (const Piece &p : pcs) {
        if (p.s == p.e) {
            const int64_t v = sc[0]++;
            out.vdest[v] = p.d * 2;
            out.vrow_ptr[v] = (int32_t)nc[0];
            continue;
        }
        int64_t last = -1;
        for (int32_t j = p.s; j < p.e; ++j) {
            const int64_t w = col[j] / W;
            if (w != last) {
                const int64_t v = sc[w]++;
                out.vdest[v] = p.d * 2 + (last >= 0 ? 1 : 0);
                out.vrow_ptr[v] = (int32_t)nc[w];
                last = w;
            }
            out.perm[nc[w]++] = j;
        }
    }
    out.vrow_ptr[nseg] = (int32_t)nz_off[nwin];
    out.win_blk.push_back(0);
    for (int w = 0; w < nwin; ++w) {
        pack_blocks(out.vrow_ptr, seg_off[w], seg_off[w + 1], cap, out, true, max_rows);
        out.win_blk.push_back((int)out.blk.size());
    }
    out.win_v = seg_off;
}

// Column-window policy (measured on MI355X; profiles/r01_windows_*.log).  A launch gathers one B row
// (kw*s bytes, at least one 128-byte L2 line) per nonzero.  Processed in row order, consecutive rows sweep a band of
// columns together, so the B lines in use at any moment are about one row span (max col - min col) wide: when the
// span's lines fit an XCD's L2 (x = span lines / L2 < 1.5; < 3 for B rows of >= 256 bytes) the plain launch already
// gathers from L2 and windows only
// add launches and C round trips (72 K rows, 500 nnz, x = 1.4: 0.58 -> 0.60..0.66 ms; 100 nnz/row, bw 0.05:
// 0.18 -> 0.30 ms).  When the span is wider, windows that keep an L2-sized slice of B hot pay, provided a row's
// piece of one window stays long (>= 48 nonzeros): 500 nnz/row matrices 1.12-1.49x at K=32 and 1.54-1.96x at K=8;
// config 2 (20 nnz over a 300 K-column span: 9 nnz per segment) and 100 nnz/row, bw 0.3 (7-27) lose 1.3-2.5x, as does
// K=1 (its 8-byte gathers are request-bound).  Returns the window width in columns, 0 = no windows.
constexpr double WIN_L2_BYTES = 4.0 * (1 << 20);   // L2 per XCD
constexpr double WIN_MIN_SPAN_NARROW = 1.5;        // row-span lines >= this many L2s, B rows <= 128 bytes
constexpr double WIN_MIN_SPAN_WIDE = 3.0;          // ... B rows >= 256 bytes (K=128 unpanelled: x 1.6-1.8 lose, >= 3.4 win)
constexpr double WIN_MIN_SEG = 48.0;               // mean nonzeros per segment at the chosen width
constexpr double WIN_MIN_ROW_BYTES = 32.0;         // B row bytes: K=1..3 fp64 gathers are request-bound
constexpr double WIN_LINE = 128.0;                 // L2 line
constexpr double WIN_MIN_LAUNCH_NNZ = 1.0e6;       // nonzeros per window launch (~500 blocks: 4 K-row rail4284 in
                                                   // 45 windows ran 120-block launches, 4x slower than one launch)
// Tiny B rows (K = 1..2 fp64, srow <= 16 B): a gather fetches a whole line for 8-16 useful bytes while continuing
// a chain into the next window costs a 2*srow C round trip, so windows pay even at ~1 nonzero per segment -- but
// only for sparse rows whose span holds more B than 1.5 L2s and while there are few windows (each launch runs a
// slice of every row) and consecutive rows do not share columns: measured (profiles/r01_s22_k1_windows,
// r01_s23_tiny_windows) 1.14-1.25x at 3-10 windows of 4 MB (1.4-4.8 M rows, bw 0.6, crs 0.05), 0.84-0.91x at
// 26-36 windows, config 2 (span 2.4 MB at K=1) 0.83x, crs 0.5-0.95 rows 0.6-0.76x.
constexpr double WIN_TINY_ROW_BYTES = 16.0;
constexpr double WIN_TINY_BYTES = 4.0 * (1 << 20);
constexpr double WIN_TINY_MAX_WINDOWS = 12.0;
constexpr double WIN_TINY_MAX_ROW = 32.0;          // mean row length (longer rows: vector lanes instead)
constexpr double WIN_TINY_MAX_CRS = 0.25;          // similar consecutive rows already share their lines in L1/L2:
                                                   // windows cost 0.6-0.76x there (profiles/r01_s23_tiny_windows/
                                                   // sweep_s160_k12_ungated.jsonl, crs 0.5-0.95)

// Window width in B bytes for a B row of srow bytes (measured best: 1-1.5 MB at K=8 fp64, 4-6 MB at K=32/128 fp64).
double window_bytes(double srow) {
    return srow <= 64.0 ? 1.5 * (1 << 20) : srow <= 128.0 ? 3.0 * (1 << 20) : 6.0 * (1 << 20);
}

// Vector lanes (measured): worth it when a staged block fills <= 1/8 of its row groups with rows of
// several gather batches -- 500 nnz/row: K=1 4.3-5x (2.20 -> 0.49 ms, 0.29 -> 0.059 ms), K=8 2x; 100 nnz/row K=1
// 1.25x -- and not above (config 2 K=1, fill 0.4: 1.00x; 100 nnz/row K=8, fill 0.31: 0.93x; 500 nnz/row K=32, fill
// 0.25: 0.65-0.99x), where it would only give up exact rows.
constexpr double VL_ROW_FILL = 0.125;
// paired short rows (spmm_kernels.hpp rows_pair_step), policy: fp64 (fp32 K = 32 measured neutral),
// mean virtual-row length at most PAIR_MAX_ROW nonzeros, at least two rows per row group, row groups of at most
// PAIR_MAX_G lanes (K <= 32: 64-lane groups lost up to 10 %), at least PAIR_MIN_NNZ nonzeros (smaller launches lost
// up to 8 %), and neighbouring rows that share columns (sampled reuse of 16-row windows, nonzeros per distinct
// column, at least PAIR_MIN_REUSE: rows with nothing in common gained nothing).  Fitted on 19 avg-5 lines, checked
// on 60 others (profiles/r06/pair/).
constexpr double PAIR_MAX_ROW = 6.0;
constexpr int PAIR_MAX_G = 16;
constexpr double PAIR_MIN_REUSE = 2.0;
constexpr int PAIR_WINDOW_ROWS = 16;
constexpr int64_t PAIR_MIN_NNZ = 4 << 20;
constexpr double VL_MIN_ROW = 32.0;   // mean virtual-row length (2 gather batches): tiny matrices stay exact

// XCD-contiguous block order (policy).  The B rows an XCD's L2 must hold at a time are about one row span (the band
// every row in flight sweeps) plus the rows in flight themselves: in the default round-robin order every XCD sees
// the rows in flight of the whole chip (~1024 resident workgroups x rows per block), in XCD order only its own
// eighth.  The order pays when that eighth brings the working set under an L2 while the chip-wide one is well
// above it -- rows of span << rows in flight (400 K rows, bw 0.01, K=32: 0.172 -> 0.154 ms) -- and only while all
// of B fits the aggregate L2 (medium sample: B <= 17 MB 1.02-1.81x, e.g. 12 K rows K=128 0.125 -> 0.069 ms; B 35-57
// MB 0.89-0.94x).  For spans wider than the rows in flight it costs 6-12 % (config 2 K=1/8/32; bw 0.05-0.3 K=1).
constexpr double XCD_RESIDENT_BLOCKS = 1024.0;   // 256 CUs x 4 workgroups (VGPR-limited occupancy)
constexpr double XCD_MAX_B_BYTES = 24.0 * (1 << 20);
bool xcd_order(const spmm_hip_t *h, double srow, double span, int cap) {
    const int64_t env = env_int("SPMM_HIP_XCD", 0);
    const int64_t forced = h->var.xcd != 0 ? h->var.xcd : env;
    if (forced != 0) return forced > 0;
    if (h->m < 8 * 64 || h->nnz == 0 || (double)h->ncols * srow > XCD_MAX_B_BYTES) return false;
    const double avg = (double)h->nnz / (double)h->m;
    const double rows_per_block = std::min((double)CAP_ROWS, std::max(1.0, (double)cap / std::max(avg, 1.0)));
    const double in_flight = std::min((double)h->m, XCD_RESIDENT_BLOCKS * rows_per_block) * (double)h->ncols / (double)h->m;
    const double line = std::max(srow, 8.0);
    return (span + in_flight / 8.0) * line <= WIN_L2_BYTES && (span + in_flight) * line > 1.5 * WIN_L2_BYTES;
}

double mean_row_span(const int32_t *rp, const int32_t *col, int64_t m) {
    double sum = 0.0;
    int64_t n = 0;
    for (int64_t r = 0; r < m; ++r)
        if (rp[r + 1] > rp[r]) {
            sum += (double)col[rp[r + 1] - 1] - (double)col[rp[r]] + 1.0;
            ++n;
        }
    return n > 0 ? sum / (double)n : 0.0;
}

// Consecutive-row similarity on a sample of row pairs: mean over rows r (non-empty, with a non-empty row r+1) of the
// fraction of r's nonzeros that have one within +-1 column in row r+1 -- the reference feature extractor's
// cross_row_similarity (csr_util_gen.c:553-610) on <= 8192 evenly spaced rows.  High similarity means a row's B
// rows were just gathered by its neighbour (L1/L2 hits); low means every nonzero gathers a fresh B row.
double row_similarity_sample(const int32_t *rp, const int32_t *col, int64_t m) {
    const int64_t ns = std::min<int64_t>(8192, m - 1);
    double sum = 0.0;
    int64_t n = 0;
    std::vector<int32_t> a, b;
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t r = i * (m - 1) / std::max<int64_t>(ns, 1);
        const int64_t la = rp[r + 1] - rp[r], lb = rp[r + 2] - rp[r + 1];
        if (la == 0 || lb == 0 || la > 4096 || lb > 4096) continue;
        a.assign(col + rp[r], col + rp[r + 1]);
        b.assign(col + rp[r + 1], col + rp[r + 2]);
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        int64_t hit = 0;
        size_t q = 0;
        for (int32_t c : a) {
            while (q < b.size() && b[q] < c - 1) ++q;
            hit += (q < b.size() && b[q] <= c + 1);
        }
        sum += (double)hit / (double)la;
        ++n;
    }
    return n > 0 ? sum / (double)n : 0.0;
}

// 128-byte K panels for gather-bound rows without cross-row reuse (measured, DESIGN §6.6, profiles/r01_s21_*): with
// 256-B B rows every nonzero of a low-similarity row gathers a fresh row, and when the rows' span holds 4-12 L2s of
// B, halving the B row halves that working set and the extra A pass is cheaper than the L2 misses it saves
// (1.06-1.25x on 1.5 M x 100 bw 0.05, 1.8 M x 20 bw 0.05, 389 K x 50 bw 0.3 at K=32 and K=128); wider or narrower
// spans, similar rows (crs >= 0.5: 0.75-0.9x) and short rows lose.
constexpr double NARROW_MAX_CRS = 0.25;
constexpr double NARROW_MIN_SPAN_L2 = 4.0, NARROW_MAX_SPAN_L2 = 12.0;
constexpr double NARROW_MIN_ROW = 20.0;

int64_t window_cols(const spmm_hip_t *h, int kw, const std::vector<Piece> &pcs, const int32_t *col,
                    int64_t win_bytes_var, double crs, int64_t *nseg_out) {
    *nseg_out = 0;
    const double srow = (double)kw * (double)h->vsize;
    const int64_t env_bytes = (int64_t)env_int("SPMM_HIP_WIN_BYTES", 0);
    const int64_t forced = win_bytes_var != 0 ? win_bytes_var : env_bytes;
    if (forced < 0 || h->nnz == 0 || h->ncols < 2) return 0;
    const bool tiny = srow <= WIN_TINY_ROW_BYTES;
    const double wb = forced > 0 ? (double)forced : tiny ? WIN_TINY_BYTES : window_bytes(srow);
    const int64_t W = std::max<int64_t>(1, (int64_t)(wb / srow));
    if (W >= h->ncols) return 0;
    if (forced == 0 && tiny) {
        const double nwin = std::ceil((double)h->ncols / (double)W);
        const double avg = (double)h->nnz / (double)std::max<int64_t>(h->m, 1);
        if (nwin > WIN_TINY_MAX_WINDOWS || avg >= WIN_TINY_MAX_ROW || crs >= WIN_TINY_MAX_CRS ||
            (double)h->nnz < WIN_MIN_LAUNCH_NNZ * nwin ||
            mean_row_span(h->h_row_ptr.data(), col, h->m) * srow < WIN_MIN_SPAN_NARROW * WIN_L2_BYTES)
            return 0;
        *nseg_out = count_segments(pcs, col, W);
        return W;
    }
    if (forced == 0) {
        if (srow < WIN_MIN_ROW_BYTES) return 0;
        const double min_span = srow <= 128.0 ? WIN_MIN_SPAN_NARROW : WIN_MIN_SPAN_WIDE;
        if (mean_row_span(h->h_row_ptr.data(), col, h->m) * std::max(srow, WIN_LINE) < min_span * WIN_L2_BYTES)
            return 0;
    }
    const int64_t nseg = count_segments(pcs, col, W);
    *nseg_out = nseg;
    if (forced > 0) return W;
    const double nwin = std::ceil((double)h->ncols / (double)W);
    if ((double)h->nnz < WIN_MIN_LAUNCH_NNZ * nwin) return 0;
    return (double)h->nnz >= WIN_MIN_SEG * (double)nseg ? W : 0;
}

// ---------------------------------------------------------------------------------------------- LDS B tiles
// TILE mode (spmm_tile_kernel).  A tile is up to rmax consecutive rows of at most T nonzeros; its
// REUSE is nnz / |union of its columns| -- how many times a B row staged in LDS is read.  The row kernel gathers
// one B row per nonzero through L1/L2 (~15 TB/s chip-wide even at 92 % L2 hits); a tile stages each
// B row of its union once and reads it from LDS.  Tiles whose reuse is below min_reuse stay with the row kernel
// (the residual rows).  Chunks: the union is cut into pieces of <= uc columns and <= capa nonzeros.

int tile_rpg(int g) { return std::max(1, std::min(8, TILE_RMAX / (WG / g))); }

// Union columns a tile may hold (the kernel keeps them in LDS): the kernel's own constexpr for its template shape.
template <typename T, int G>
int tile_colmax_t() {
    constexpr int NG = WG / G;
    constexpr int RPG = NG * 8 <= TILE_RMAX ? 8 : (TILE_RMAX / NG > 1 ? TILE_RMAX / NG : 1);
    return tile_colmax<T, 16 / (int)sizeof(T), G, TILE_UCB, TILE_CAPA, NG * RPG>();
}
int tile_colmax_for(size_t vsize, int g) {
    auto pick = [&](auto t) -> int {
        using T = decltype(t);
        switch (g) {
            case 4: return tile_colmax_t<T, 4>();
            case 8: return tile_colmax_t<T, 8>();
            case 16: return tile_colmax_t<T, 16>();
            case 32: return tile_colmax_t<T, 32>();
            default: return tile_colmax_t<T, 64>();
        }
    };
    return vsize == 8 ? pick(0.0) : pick(0.0f);
}

struct TilePlan {
    std::vector<int4> tiles;       // {first row, rows, first chunk, chunks}
    std::vector<int4> chunks;      // {first tcol, columns, first nonzero (8-aligned), first tseg (8-aligned)} + sentinel
    std::vector<int32_t> tcol;     // union columns, chunk by chunk
    std::vector<uint16_t> tseg;    // per chunk: rows+1 segment offsets (relative to the chunk's first nonzero)
    std::vector<int64_t> perm;     // chunk-major position -> original nonzero (-1: alignment padding)
    std::vector<uint16_t> tlidx;   // chunk-major position -> chunk-local column
    std::vector<uint8_t> in_tile;  // per row
    int64_t rows = 0, nnz = 0;
};

// Reuse of rows [r0, r1): nnz / distinct columns (stamp/epoch marking; 0 for an empty range).  Stops counting once
// the union makes the reuse fall below `floor` (returns what it has, which is then < floor).
double tile_reuse(const int32_t *rp, const int32_t *col, int64_t r0, int64_t r1, std::vector<int32_t> &stamp,
                  int32_t epoch, double floor, int64_t *nu_out) {
    const int64_t nnz = (int64_t)rp[r1] - rp[r0];
    int64_t nu = 0;
    const int64_t nu_max = floor > 0 ? (int64_t)((double)nnz / floor) + 1 : INT64_MAX;
    for (int64_t j = rp[r0]; j < rp[r1]; ++j) {
        const int32_t c = col[j];
        if (stamp[(size_t)c] != epoch) {
            stamp[(size_t)c] = epoch;
            if (++nu > nu_max) break;
        }
    }
    if (nu_out) *nu_out = nu;
    return nu > 0 ? (double)nnz / (double)nu : 0.0;
}

// Build the tiles.  A run of up to rmax consecutive rows of <= T nonzeros is a candidate; it becomes a tile when
// its reuse is >= min_reuse, no column repeats more often than a chunk holds, its union fits the kernel's LDS column
// list (<= colmax) and it makes <= dmax chunks -- a candidate over the last two is halved until it fits.  Rows must
// be sorted (checked by the caller).  Returns false when no tile qualifies.
bool build_tiles(const int32_t *rp, const int32_t *col, int64_t m, int64_t ncols, int T, int rmax, int uc, int capa,
                 double min_reuse, TilePlan &tp, int colmax = INT32_MAX, int dmax = INT32_MAX,
                 double min_npc = 0.0) {
    tp = TilePlan();
    tp.in_tile.assign((size_t)m, 0);
    std::vector<int32_t> stamp((size_t)ncols, -1), pos((size_t)ncols, 0);
    std::vector<int32_t> ulist, cnt;
    int32_t epoch = 0;
    auto next_epoch = [&]() {
        if (epoch == INT32_MAX) {
            std::fill(stamp.begin(), stamp.end(), -1);
            epoch = 0;
        }
        return ++epoch;
    };
    auto eligible = [&](int64_t r) { return (int64_t)rp[r + 1] - rp[r] <= T; };
    enum { TAKE, SKIP, SHRINK };
    // evaluate (and on TAKE append) rows [r, r1)
    auto attempt = [&](int64_t r, int64_t r1) -> int {
        const int64_t nnz = (int64_t)rp[r1] - rp[r];
        int64_t nu = 0;
        const double reuse = tile_reuse(rp, col, r, r1, stamp, next_epoch(), min_reuse, &nu);
        if (nnz == 0 || reuse < min_reuse) return SKIP;
        // sorted union, local positions, per-column counts
        ulist.clear();
        const int32_t ep = next_epoch();
        for (int64_t j = rp[r]; j < rp[r1]; ++j)
            if (stamp[(size_t)col[j]] != ep) stamp[(size_t)col[j]] = ep, ulist.push_back(col[j]);
        if ((int64_t)ulist.size() > colmax) return SHRINK;
        std::sort(ulist.begin(), ulist.end());
        cnt.assign(ulist.size(), 0);
        for (size_t u = 0; u < ulist.size(); ++u) pos[(size_t)ulist[u]] = (int32_t)u;
        const int nrows = (int)(r1 - r);
        const int64_t room = capa - (int64_t)nrows * (TILE_SEG_ALIGN - 1);   // each row's padding (< 4 entries)
        bool ok = room > 0;
        for (int64_t j = rp[r]; j < rp[r1] && ok; ++j) ok = ++cnt[(size_t)pos[(size_t)col[j]]] <= room;
        if (!ok) return nrows > 1 ? SHRINK : SKIP;
        // chunk boundaries over the sorted union: <= uc columns and <= room entries
        std::vector<size_t> cut{0};
        for (size_t u0 = 0; u0 < ulist.size();) {
            size_t u1 = u0;
            int64_t cz = 0;
            while (u1 < ulist.size() && (int64_t)(u1 - u0) < uc && (u1 == u0 || cz + cnt[u1] <= room)) cz += cnt[u1++];
            cut.push_back(u1);
            u0 = u1;
        }
        if ((int64_t)cut.size() - 1 > dmax) return SHRINK;
        // matrix-core tiles: a tile must bring enough nonzeros per chunk (per dense panel product) to beat the row
        // kernel on its rows (mfma_cost); otherwise its rows stay with the row kernel
        if ((double)nnz < min_npc * (double)(cut.size() - 1)) return SKIP;
        const int c_first = (int)tp.chunks.size();
        std::vector<int32_t> rowp(rp + r, rp + r1);     // per row: next nonzero not yet placed
        for (size_t ci = 0; ci + 1 < cut.size(); ++ci) {
            const size_t u0 = cut[ci], u1 = cut[ci + 1];
            int4 ch;
            ch.x = (int)tp.tcol.size();
            ch.y = (int)(u1 - u0);
            ch.z = (int)tp.perm.size();
            ch.w = (int)tp.tseg.size();
            tp.tcol.insert(tp.tcol.end(), ulist.begin() + (ptrdiff_t)u0, ulist.begin() + (ptrdiff_t)u1);
            int32_t off = 0;
            for (int q = 0; q < nrows; ++q) {
                tp.tseg.push_back((uint16_t)off);
                int32_t &p = rowp[(size_t)q];
                const int32_t pe = rp[r + q + 1];
                while (p < pe && (size_t)pos[(size_t)col[p]] < u1) {
                    tp.perm.push_back(p);
                    tp.tlidx.push_back((uint16_t)(pos[(size_t)col[p]] - (int32_t)u0));
                    ++p, ++off;
                }
                while (off % TILE_SEG_ALIGN) tp.perm.push_back(-1), tp.tlidx.push_back(TILE_PAD_LIDX), ++off;
            }
            tp.tseg.push_back((uint16_t)off);
            while (tp.tseg.size() % 8) tp.tseg.push_back((uint16_t)off);
            while (tp.perm.size() % 8) tp.perm.push_back(-1), tp.tlidx.push_back(0);
            tp.chunks.push_back(ch);
        }
        tp.tiles.push_back(make_int4((int)r, nrows, c_first, (int)tp.chunks.size() - c_first));
        for (int64_t q = r; q < r1; ++q) tp.in_tile[(size_t)q] = 1;
        tp.rows += nrows;
        tp.nnz += nnz;
        return TAKE;
    };
    int64_t r = 0;
    while (r < m) {
        if (!eligible(r)) {
            ++r;
            continue;
        }
        int64_t r1 = r;
        while (r1 < m && r1 - r < rmax && eligible(r1)) ++r1;
        int st;
        while ((st = attempt(r, r1)) == SHRINK && r1 - r > 1) r1 = r + (r1 - r) / 2;
        r = r1;
    }
    tp.chunks.push_back(make_int4((int)tp.tcol.size(), 0, (int)tp.perm.size(), (int)tp.tseg.size()));
    return !tp.tiles.empty();
}

// The tile tables are addressed with 32-bit positions (chunk descriptors' first entry / column / segment, the
// kernel's tval + ch.z, d_tperm): every padded table must stay below 2^31 entries.  Each row segment is padded to
// 4 entries in every chunk it touches, so the padded count can be well above nnz (a ~1.3e9-nonzero short-row
// matrix would overflow).  SPMM_HIP_TILE_INDEX_LIMIT lowers the limit (tests of this guard only).
int64_t tile_index_limit() {
    const char *v = getenv("SPMM_HIP_TILE_INDEX_LIMIT");
    const long long l = (v && *v) ? atoll(v) : 0;
    return l > 0 ? std::min<int64_t>(l, INT32_MAX) : (int64_t)INT32_MAX;
}
bool tile_tables_fit(const TilePlan &tp) {
    const int64_t lim = tile_index_limit(), pad = PAD_BYTES;
    return (int64_t)tp.perm.size() + pad < lim && (int64_t)tp.tseg.size() + pad < lim &&
           (int64_t)tp.tcol.size() + pad < lim && (int64_t)tp.chunks.size() < lim;
}

// Policy gate: mean reuse over <= 256 evenly spaced candidate tiles (cheap; the full build only runs when tiles can
// pay).  Returns the sampled mean reuse.
double tile_reuse_sample(const int32_t *rp, const int32_t *col, int64_t m, int64_t ncols, int T, int rmax) {
    if (m == 0) return 0.0;
    std::vector<int32_t> stamp((size_t)ncols, -1);
    const int64_t ntiles = (m + rmax - 1) / rmax;
    const int64_t ns = std::min<int64_t>(256, ntiles);
    double sum = 0.0;
    int64_t n = 0;
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t t = i * ntiles / ns;
        const int64_t r0 = t * rmax, r1 = std::min<int64_t>(m, r0 + rmax);
        bool ok = true;
        for (int64_t r = r0; r < r1 && ok; ++r) ok = (int64_t)rp[r + 1] - rp[r] <= T;
        if (!ok || rp[r1] == rp[r0]) continue;
        sum += tile_reuse(rp, col, r0, r1, stamp, (int32_t)i, 0.0, nullptr);
        ++n;
    }
    return n > 0 ? sum / (double)n : 0.0;
}

// ------------------------------------------------------------------------------------ matrix-core policy (gate)
// Whether a matrix runs its dense 16-row tiles on the matrix cores.  Decided from a sample of
// MFMA_GATE_SAMPLE evenly spaced 16-row candidate tiles -- the gate reads the columns of those rows only (so a
// census of the whole medium dataset can evaluate it from the sampled rows, tools/plan_census.py) -- plus m, nnz and
// the panel shape: per sampled tile its nonzeros, union columns and the chunks build_tiles would cut; the taken ones
// (reuse >= MFMA_TILE_REUSE) scaled to the matrix give the work of the tile kernel and of the row kernel on the same
// rows, priced by mfma_cost (measured constants).
constexpr int MFMA_GATE_SAMPLE = 256;
// The cost model (us; GateModel below, fitted on same-process A/B data by tools/fit_mfma_gate.py, DESIGN §6.18,
// §6.22).  Per 32-column sub-panel the tile kernel streams each chunk's B rows and MFMAs at a chip-wide rate
// (us_chunk per chunk, us_tile per tile for its prologue / epilogue) unless it has too few tiles to fill the chip,
// when the longest tile's chunk chain bounds it (us_chain per chunk); each launch also checks B's exact range (us_bmb
// per MB of B).  The row kernel gathers one B row per nonzero per sub-panel (row_nnz, cheaper for similar rows -- L2
// hits -- and for unpanelled launches that read A once for all columns) plus a per-row cost (C store, row setup).  A
// tile is taken when it brings at least `npc` nonzeros per chunk; a matrix takes matrix-core tiles when they hold
// min_tile_frac of its nonzeros and the model's time with them (tiles beside the leftover rows) beats the row
// kernel's by min_gain.
// One constant set per value type (the matrix-core tile kernel, its B operand and the row kernel's gather all differ
// in width between fp64 and fp32).  `on` = false: the default policy never takes matrix-core tiles for that type
// (SPMM_HIP_MFMA >= 1 still does).
struct GateModel {
    double us_chunk, us_tile, us_chain, us_launch;     // tile kernel
    double us_bmb;           // + the per-launch exact-range check of B, per MB of B
    double row_launch, row_nnz, row_reuse_exp, row_kw_exp, row_row;   // row kernel
    double npc;              // nonzeros per chunk for a tile to be taken (MFMA_TILE_NPC)
    double min_tile_frac;    // taken tiles must hold this share of the nonzeros
    double min_gain;         // model gain the gate asks for
    double k32_min_row_nnz;  // one 32-column sub-panel (K < 64): rows must average this many nonzeros
    bool on;
};
// Round-5 fits (tools/fit_mfma_gate.py on same-process A/B of the gate forced open against no matrix-core tiles, the
// round-5 tile kernel, 168 lines x K 32 / 128 per type, profiles/r05/fit/).  Rule per type from the
// fit sample: taken tiles hold >= 90 % of the nonzeros and the model gains >= 1.2x (fp64: 48 pairs taken, worst
// 1.05x, aggregate 1.11x; fp32: 36 taken, worst 1.00x, aggregate 1.06x).  K < 64 rule (rows averaging < 32
// nonzeros keep the row kernel at one 32-column sub-panel): the round-4 changed-lines sweep measured avg-10 / avg-20
// lines at K = 32 at 0.79x / 0.95x alone on the GPU.
constexpr GateModel GATE_F64 = {0.001271, 0.001405, 0.9645, 27.58, 0.1616, 6.283, 1.582e-05,
                                0.04599, 0.2127, 7.99e-05, 96.0, 0.9, 1.2, 32.0, true};
constexpr GateModel GATE_F32 = {0.0007035, 0.0, 0.6146, 31.06, 0.519, 6.935, 7.987e-06,
                                -0.0298, 0.1672, 3.012e-05, 96.0, 0.9, 1.2, 32.0, true};
inline const GateModel &gate_model(size_t vsize) { return vsize == 8 ? GATE_F64 : GATE_F32; }
constexpr int64_t MFMA_GATE_MIN_NNZ = 500000;
struct MfmaGate {
    int sampled = 0;          // candidate tiles sampled (all rows <= T, not empty)
    double r16 = 0.0;         // mean reuse of the sampled tiles (nonzeros per union column)
    double take = 0.0;        // fraction of sampled tiles the build would take
    double tiles = 0.0;       // estimated taken tiles (whole matrix)
    double tile_nnz = 0.0;    // estimated nonzeros in taken tiles (whole matrix)
    double chunks = 0.0;      // estimated chunks of the taken tiles (whole matrix)
    double max_chunks = 0.0;  // largest chunk count of a sampled taken tile
    double t_on = 0.0, t_off = 0.0;   // cost model (us): tiles beside the leftover rows vs the row kernel alone
    int verdict = 0;          // 1 = matrix-core tiles
};

// chunks build_tiles cuts for a tile of nnz entries over nu union columns: <= MFMA_UC columns and <= room entries
inline double mfma_chunks_est(double nnz, double nu) {
    const double room = MFMA_CAPA - (double)MFMA_ROWS * (TILE_SEG_ALIGN - 1);
    return std::max(std::ceil(nu / MFMA_UC), std::ceil(nnz / room));
}

// The gate's sample: f(i, r0, r1) for the rows [r0, r1) of sampled candidate tile i (spmm_amd.gate_sample_rows is
// the same list)
template <typename F>
void mfma_gate_tiles(int64_t m, F f) {
    const int64_t ntiles = (m + MFMA_ROWS - 1) / MFMA_ROWS;
    const int64_t ns = std::min<int64_t>(MFMA_GATE_SAMPLE, ntiles);
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t t = i * ntiles / ns;
        const int64_t r0 = t * MFMA_ROWS;
        f(i, r0, std::min<int64_t>(m, r0 + MFMA_ROWS));
    }
}

MfmaGate mfma_sample(const int32_t *rp, const int32_t *col, int64_t m, int64_t ncols, int T, double min_reuse,
                     double min_npc) {
    MfmaGate g;
    if (m == 0) return g;
    std::vector<int32_t> stamp((size_t)ncols, -1);
    const int64_t ntiles = (m + MFMA_ROWS - 1) / MFMA_ROWS;
    const int64_t ns = std::min<int64_t>(MFMA_GATE_SAMPLE, ntiles);
    double sum_r = 0.0, nz_taken = 0.0, ch_taken = 0.0, n_taken = 0.0;
    mfma_gate_tiles(m, [&](int64_t i, int64_t r0, int64_t r1) {
        bool ok = true;
        for (int64_t r = r0; r < r1 && ok; ++r) ok = (int64_t)rp[r + 1] - rp[r] <= T;
        if (!ok || rp[r1] == rp[r0]) return;
        int64_t nu = 0;
        const double reuse = tile_reuse(rp, col, r0, r1, stamp, (int32_t)i, 0.0, &nu);
        sum_r += reuse;
        ++g.sampled;
        const double nnz = (double)(rp[r1] - rp[r0]);
        const double ch = mfma_chunks_est(nnz, (double)nu);
        if (reuse >= min_reuse && nnz >= min_npc * ch) {
            nz_taken += nnz, ch_taken += ch, n_taken += 1.0;
            g.max_chunks = std::max(g.max_chunks, ch);
        }
    });
    if (g.sampled == 0) return g;
    g.r16 = sum_r / g.sampled;
    g.take = n_taken / g.sampled;
    const double scale = (double)ntiles / (double)ns;   // sampled slots -> all candidate slots
    g.tiles = n_taken * scale;
    g.tile_nnz = nz_taken * scale;
    g.chunks = ch_taken * scale;
    return g;
}

// The gate: the cost model above for the K columns in 32-column sub-panels.
void mfma_cost(MfmaGate &g, int64_t m, int64_t ncols, int64_t nnz, int k, int kw, size_t vsize, const GateModel &c) {
    const double P = (double)k / 32.0;
    const double r_row = c.row_nnz * std::pow(std::max(g.r16, 1.0), -c.row_reuse_exp) *
                         std::pow((double)std::max(kw, 1) / 32.0, -c.row_kw_exp);
    g.t_off = c.row_launch + P * ((double)nnz * r_row + (double)m * c.row_row);
    const double t_tiles = c.us_launch + P * std::max(g.chunks * c.us_chunk + g.tiles * c.us_tile,
                                                      g.max_chunks * c.us_chain) +
                           c.us_bmb * (double)ncols * (double)k * (double)vsize * 1e-6;
    const double left_rows = std::max((double)m - (double)MFMA_ROWS * g.tiles, 0.0);
    const double t_left = c.row_launch + P * (((double)nnz - g.tile_nnz) * r_row + left_rows * c.row_row);
    g.t_on = std::max(t_tiles, t_left);
    g.verdict = (c.on && g.tiles > 0 && nnz >= MFMA_GATE_MIN_NNZ && g.tile_nnz >= c.min_tile_frac * (double)nnz &&
                 g.t_off >= c.min_gain * g.t_on && (k >= 64 || (double)nnz >= c.k32_min_row_nnz * (double)m))
                    ? 1 : 0;
}

// Everything the inspector decides for (matrix, K), on the host: the plan, the tile plan, the block decomposition,
// the exact-row mask and the fused-combine slot table.  spmm_hip_plan turns it into device tables;
// spmm_hip_debug_plan reports it without a device.
struct Draft {
    Plan pl;
    TilePlan tp;
    bool tiles = false;
    Inspection in;
    int64_t W = 0;
    std::vector<int32_t> slot_lr;
    bool fuse = false;
    std::vector<uint8_t> exact;
    MfmaGate gate;
    bool gate_only = false;      // stopped after the matrix-core gate (census mode, no full tile build)
};

// hcol_in: the matrix's columns on the host (nullptr: read from the handle's device copy).  gate_only: stop after
// the matrix-core gate, which reads only its sampled rows' columns (tools/plan_census.py passes a column array
// filled for those rows only).
int draft_plan(const spmm_hip_t *h, int k, const int32_t *hcol_in, bool gate_only, Draft &d) {
    Plan &pl = d.pl;
    pl = Plan();
    pl.k = k;
    // K panels of PANEL_ROW_BYTES-byte B rows when B would crowd the Infinity Cache and the B gather dominates the
    // launch (>= 16 nonzeros per row); each extra panel re-streams A and cuts C rows into 256-B pieces, which only
    // pays when it turns Infinity-Cache misses into hits (measured §6.2: config 2 K=128 1.65 ms at 32 columns vs
    // 2.30 ms unpanelled; a 200 K-row, 10 nnz/row matrix with a 208 MB B is faster unpanelled).
    const int panel_env = env_int("SPMM_HIP_PANEL_K", 0);
    const double b_bytes = (double)h->ncols * k * (double)h->vsize;
    const double avg_row = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    pl.kw = k;
    if (h->var.panel_k > 0 || panel_env > 0) {
        pl.kw = std::min(k, h->var.panel_k > 0 ? h->var.panel_k : panel_env);
    } else if (b_bytes > PANEL_MIN_B_BYTES && avg_row >= PANEL_MIN_ROW_NNZ) {
        pl.kw = std::min(k, std::max(1, (int)(PANEL_ROW_BYTES / h->vsize)));
    }
    // col_idx on the host (span, row similarity, windows, XCD order) when some policy below may need it
    std::vector<int32_t> hstore;
    const int32_t *hcol = nullptr;
    double span = (double)h->ncols, crs = 1.0;
    auto load_cols = [&]() -> int {
        if (hcol || h->nnz == 0) return SPMM_HIP_OK;
        if (hcol_in) {
            hcol = hcol_in;
        } else {
            hstore.resize((size_t)h->nnz);
            HIPCHK(hipMemcpy(hstore.data(), h->d_col, (size_t)h->nnz * 4, hipMemcpyDeviceToHost));
            hcol = hstore.data();
        }
        if (!gate_only) {
            span = mean_row_span(h->h_row_ptr.data(), hcol, h->m);
            crs = row_similarity_sample(h->h_row_ptr.data(), hcol, h->m);
        }
        return SPMM_HIP_OK;
    };
    if (!gate_only && h->var.panel_k <= 0 && panel_env <= 0 && (double)pl.kw * h->vsize == 2.0 * WIN_LINE &&
        avg_row >= NARROW_MIN_ROW && h->m > 1) {
        if (int st = load_cols()) return st;
        const double x = span * 2.0 * WIN_LINE / WIN_L2_BYTES;
        if (crs < NARROW_MAX_CRS && x >= NARROW_MIN_SPAN_L2 && x <= NARROW_MAX_SPAN_L2) pl.kw /= 2;
    }
    // small matrices: a launch of a few hundred blocks leaves most of the 256 CUs idle and its rows'
    // gather chains exposed; narrower K panels, all in ONE launch (blockIdx.y = panel), give more blocks and more
    // vector-lane groups per row.  SPMM_HIP_SMALL_KW=<cols> sets the panel width (0: off).
    {
        const int small_kw = env_int("SPMM_HIP_SMALL_KW", SMALL_KW_DEFAULT);
        if (h->var.panel_k <= 0 && panel_env <= 0 && small_kw > 0 && h->nnz > 0 && h->nnz < SMALL_NNZ &&
            pl.kw == k && k > small_kw && k % small_kw == 0)
            pl.kw = small_kw, pl.ygrid = 1;
    }
    pl.npanels = (k + pl.kw - 1) / pl.kw;
    // block capacity and split length
    int vec, g;
    lane_layout(pl.kw, k, h->vsize, vec, g);
    // block capacity: the LDS window (CAP), smaller for small matrices so >= ~1024 blocks exist (a 4096-nonzero
    // window for one-lane row groups measured slower at K = 1, §6.2)
    const int cap_env = env_int("SPMM_HIP_CAP", 0);
    // the wide window CAP_BIG only where its kernel exists (16-byte lanes, groups of >= 8 lanes, one launch per panel)
    // Policy: fp64 matrices of >= WIDE_MIN_NNZ nonzeros whose rows average >= WIDE_MIN_ROW take the
    // wide window unless column windows or tiles are chosen below (both lower it back to CAP).
    const bool big_ok = vec * (int)h->vsize == 16 && g >= 8;
    const double avg_nnz_row = h->m > 0 ? (double)h->nnz / (double)h->m : 0.0;
    const bool wide = big_ok && h->vsize == 8 && k == 32 && pl.kw == 32 && h->nnz >= WIDE_MIN_NNZ &&
                      avg_nnz_row >= WIDE_MIN_ROW;      // measured at K = 32 fp64 only (K = 128 lost, §6.43)
    pl.cap = h->var.cap > 0 ? std::min(h->var.cap, CAP)
             : cap_env > 0   ? std::min(cap_env, (cap_env > CAP && big_ok) ? CAP_BIG : CAP)
             : wide          ? CAP_BIG
                             : std::max(256, std::min(CAP, pow2_ceil(h->nnz / 1024)));
    const int seq_env = env_int("SPMM_HIP_SEQ_MAX", 0);
    pl.seq_max = h->var.seq_max > 0 ? h->var.seq_max : seq_env > 0 ? seq_env : split_length(h, pl.kw);
    pl.seq_max = std::max(1, std::min(pl.seq_max, CAP));
    pl.cap = std::max(pl.cap, std::min(CAP, pow2_ceil(pl.seq_max)));   // a row of T nonzeros fits one block
    pl.piece = pl.seq_max;
    // rows per block: one row per row group when a group's row is long (>= 64 nonzeros) and a block of NG rows fits
    // the LDS window -- the greedy packing would otherwise put NG + a few rows in a block and make a quarter of the
    // groups run two rows while the rest idle (measured K=32, avg 100: 1.03-1.13x; avg 500 blocks hold < NG rows
    // anyway; avg 20-50 unchanged or slower, r03_s2 / r03_s3 probes)
    {
        int vec_b, g_b;
        lane_layout(pl.kw, k, h->vsize, vec_b, g_b);
        const int ng = WG / g_b;
        const int env_rows = env_int("SPMM_HIP_BLOCK_ROWS", 0);
        pl.block_rows = CAP_ROWS;
        if (env_rows > 0)
            pl.block_rows = std::min(CAP_ROWS, env_rows);
        else if (avg_row >= 64.0 && (double)ng * avg_row <= (double)pl.cap)
            pl.block_rows = ng;
    }

    const int64_t srow_t = (int64_t)pl.kw * (int64_t)h->vsize;
    // LDS B tiles: rows whose union of columns is reused enough leave the row kernel.  Needs 16-byte
    // B pieces in every panel and sorted rows.  SPMM_HIP_TILES=-1 off / 1 every eligible tile; SPMM_HIP_TILE_REUSE
    // sets the policy threshold.
    TilePlan &tp = d.tp;
    bool &tiles = d.tiles;
    tiles = false;
    {
        const int64_t srow = srow_t;
        const int env_t = env_int("SPMM_HIP_TILES", 0);
        const int forced = h->var.tiles != 0 ? h->var.tiles : env_t;
        int vec_t, g_t;
        lane_layout(pl.kw, k, h->vsize, vec_t, g_t);
        const bool shape_ok = h->nnz > 0 && vec_t == (int)(16 / h->vsize) && ((int64_t)k * h->vsize) % 16 == 0 &&
                              srow % 16 == 0 && k % pl.kw == 0 && srow >= 64 && srow <= 1024 &&
                              pow2_ceil(srow / 16) == srow / 16 &&
                              h->ncols < INT32_MAX;
        const int64_t win_forced = h->var.win_bytes != 0 ? h->var.win_bytes : (int64_t)env_int("SPMM_HIP_WIN_BYTES", 0);
        // matrix-core tiles first: fp64 32-column panels, strictly increasing columns, B < 4 GiB.
        // SPMM_HIP_MFMA: -1 off, 0 policy (the gate), 1 every eligible tile of reuse >= 1, 2 the gate open with the
        // policy's per-tile threshold (what the policy runs once a matrix qualifies; A/B measurements)
        const int env_m = env_int("SPMM_HIP_MFMA", 0);
        const int fm = h->var.mfma != 0 ? h->var.mfma : env_m;
        const bool mshape = fm >= 0 && k % 32 == 0 && (double)h->ncols * (double)k * (double)h->vsize < 4294967296.0;
        if (forced >= 0 && h->nnz > 0 && h->ncols < INT32_MAX && win_forced <= 0 && (mshape || shape_ok)) {
            if (int st = load_cols()) return st;
            if (mshape && (gate_only || rows_strict(h->h_row_ptr.data(), hcol, h->m))) {
                const char *mthr = getenv("SPMM_HIP_MFMA_REUSE");
                const bool force_all = forced > 0 || fm == 1;
                const double treuse = (mthr && *mthr) ? atof(mthr) : force_all ? 1.0 : MFMA_TILE_REUSE;
                const char *npc_env = getenv("SPMM_HIP_MFMA_NPC");   // measurement override of MFMA_TILE_NPC
                const GateModel &gm = gate_model(h->vsize);
                const double npc = force_all ? 0.0 : (npc_env && *npc_env) ? atof(npc_env) : gm.npc;
                d.gate = mfma_sample(h->h_row_ptr.data(), hcol, h->m, h->ncols, pl.seq_max, treuse, npc);
                mfma_cost(d.gate, h->m, h->ncols, h->nnz, k, pl.kw, h->vsize, gm);
                pl.tile_reuse = d.gate.r16;
                if (gate_only) {
                    d.gate_only = true;
                    pl.tile_mfma = (force_all || fm == 2 || d.gate.verdict) ? 1 : 0;
                    return SPMM_HIP_OK;
                }
                if (force_all || fm == 2 || d.gate.verdict) {
                    tiles = build_tiles(h->h_row_ptr.data(), hcol, h->m, h->ncols, pl.seq_max, MFMA_ROWS,
                                        MFMA_UC, MFMA_CAPA, treuse, tp, INT32_MAX, INT32_MAX, npc);
                    if (tiles && !tile_tables_fit(tp)) tiles = false;
                    if (tiles) pl.tile_mfma = 1;
                }
            }
            if (gate_only) {        // census mode: the matrix-core gate is all it reports
                d.gate_only = true;
                return SPMM_HIP_OK;
            }
            if (!tiles && shape_ok && rows_sorted(h->h_row_ptr.data(), hcol, h->m)) {
                const int rows_env = env_int("SPMM_HIP_TILE_ROWS", 0);
                int rmax = std::min((WG / g_t) * tile_rpg(g_t), rows_env > 0 ? rows_env : TILE_ROWS);
                const char *thr = getenv("SPMM_HIP_TILE_REUSE");
                const double min_reuse = forced > 0 ? 1.0 : (thr && *thr) ? atof(thr) : TILE_MIN_REUSE;
                pl.tile_reuse = tile_reuse_sample(h->h_row_ptr.data(), hcol, h->m, h->ncols, pl.seq_max, rmax);
                const bool enough = (h->m + rmax - 1) / rmax >= TILE_MIN_TILES && srow <= TILE_POLICY_MAX_ROW;
                if (forced > 0 || (enough && pl.tile_reuse >= min_reuse))
                    tiles = build_tiles(h->h_row_ptr.data(), hcol, h->m, h->ncols, pl.seq_max, rmax,
                                        (int)(TILE_UCB / srow), TILE_CAPA, min_reuse, tp,
                                        tile_colmax_for(h->vsize, g_t) - 4, TILE_DMAX - 1);
                if (tiles && forced <= 0 && (int64_t)tp.tiles.size() < TILE_MIN_BUILT) tiles = false;
                if (tiles && !tile_tables_fit(tp)) tiles = false;     // 32-bit tile positions (row kernel instead)
            }
        }
        if (gate_only) {
            d.gate_only = true;
            return SPMM_HIP_OK;
        }
        if (tiles) {
            pl.ntile = (int)tp.tiles.size();
            pl.tile_rows = tp.rows;
            pl.tile_nnz = tp.nnz;
            pl.tile_chunks = (int64_t)tp.chunks.size() - 1;
            // consecutive tiles share most of their columns: in XCD order they share an L2 as well
            const int env_x = env_int("SPMM_HIP_TILE_XCD", 1);
            pl.tile_xcd = (env_x > 0 && pl.ntile >= 64) ? 1 : 0;
            // compute-lane width in 16-byte pieces: the requested 1/2/4, lowered until rows per group divide
            int sw = std::max(1, env_int("SPMM_HIP_TILE_WIDE", TILE_WIDE_DEFAULT));
            sw = sw >= 2 ? 2 : 1;
            while (sw > 1 && tile_rpg(g_t) % sw != 0) sw /= 2;
            pl.tile_wide = sw;
        } else {
            pl.tile_mfma = 0;
        }
    }

    // XCD-contiguous order, else column windows (chained mode; needs every row's columns sorted); both decided from
    // col_idx on the host
    Inspection &in = d.in;
    int64_t &W = d.W;
    W = 0;
    {
        const double srow = (double)pl.kw * (double)h->vsize;
        const int64_t env_bytes = (int64_t)env_int("SPMM_HIP_WIN_BYTES", 0);
        const int64_t forced = h->var.win_bytes != 0 ? h->var.win_bytes : env_bytes;
        const bool b_big = (double)h->ncols * std::max(srow, WIN_LINE) > WIN_MIN_SPAN_NARROW * WIN_L2_BYTES;
        const bool maybe_win = h->nnz > 0 && forced >= 0 && (forced > 0 || (b_big && (srow >= WIN_MIN_ROW_BYTES || srow <= WIN_TINY_ROW_BYTES)));
        const bool maybe_xcd = h->nnz > 0 && (double)h->ncols * srow > WIN_L2_BYTES;
        if (maybe_win || maybe_xcd) {
            if (int st = load_cols()) return st;
        }
        pl.xcd = xcd_order(h, srow, span, pl.cap) ? 1 : 0;
        if (!tiles && maybe_win && forced >= 0 && (forced > 0 || !pl.xcd) &&
            rows_sorted(h->h_row_ptr.data(), hcol, h->m)) {
            std::vector<Piece> pcs;
            Inspection tmp;
            make_pieces(h->h_row_ptr.data(), h->m, pl.seq_max, pcs, tmp);
            W = window_cols(h, pl.kw, pcs, hcol, h->var.win_bytes, crs, &pl.nseg);
        }
    }
    // the wide window only for the plain row kernel: column windows (chained mode) and the tiles' leftover rows keep
    // the default one (the wide window measured 0.70-0.82x where it displaced column windows, §6.43)
    if ((W > 0 || tiles) && pl.cap > CAP) pl.cap = CAP;
    if (W > 0) {
        pl.xcd = 0;
        inspect_windows(h->h_row_ptr.data(), hcol, h->m, h->ncols, pl.seq_max, pl.cap, W, in, pl.block_rows);
        pl.win_cols = W;
        pl.nwin = (int)in.win_blk.size() - 1;
        pl.nseg = (int64_t)in.vdest.size();
    } else {
        // when tiles hold nearly all the work, the row kernel's launch is only the leftover rows -- typically one
        // skewed row of thousands of nonzeros whose T-pieces each run as a latency-bound serial chain (~64 us for
        // 2,048 gathers) after the tile kernel: the rows longer than T are cut into GAP_SEQ_MAX-nonzero pieces
        // instead (rows of <= T nonzeros stay whole, one exact chain)
        if (tiles && pl.tile_mfma && (double)(h->nnz - tp.nnz) < GAP_SHORT_FRAC * (double)h->nnz &&
            pl.seq_max > GAP_SEQ_MAX && h->var.seq_max <= 0 && env_int("SPMM_HIP_SEQ_MAX", 0) <= 0)
            pl.piece = GAP_SEQ_MAX;
        inspect(h->h_row_ptr.data(), h->m, pl.seq_max, pl.cap, in, /*heavy_first=*/!pl.xcd,
                tiles ? tp.in_tile.data() : nullptr, pl.block_rows, pl.piece);
        pl.nseg = (int64_t)in.vrow_ptr.size() - 1;
    }
    const int nblk = (int)in.blk.size();
    // one-launch panels: not with column windows (separate launches then); split rows are combined by the separate
    // combine kernel afterwards (the fused combine counts one row's pieces within one panel)
    if (pl.ygrid && (W > 0 || k % pl.kw != 0)) pl.ygrid = 0;
    // vector lanes when the staged blocks hold fewer rows than row groups (long rows at small K), and
    // the exact-row mask: rows <= T whose every virtual row sits in a block with L = 1
    {
        int vec, g;
        lane_layout(pl.kw, k, h->vsize, vec, g);
        const int ng = WG / g;
        const int lcap = std::max(1, 64 / g);
        // the rows the row kernel runs: gap virtual rows and the tile rows' nonzeros are not among them
        const double nvr = (double)((int64_t)in.vrow_ptr.size() - 1 - in.ngaps);
        const double nnz_rows = (double)(h->nnz - (tiles ? tp.nnz : 0));
        const double rows_per_block = in.blk.empty() ? 0.0 : nvr / (double)nblk;
        const double mean_vrow = nvr > 0 ? nnz_rows / nvr : 0.0;
        const int env_l = env_int("SPMM_HIP_LANES", 0);
        const int forced = h->var.lanes != 0 ? h->var.lanes : env_l;
        bool all_blocks = false;
        if (forced != 0)
            all_blocks = forced > 0, pl.lmax = forced > 0 ? std::min(forced, lcap) : 1;
        else
            all_blocks = nnz_rows > 0 && rows_per_block <= VL_ROW_FILL * ng && mean_vrow >= VL_MIN_ROW,
            pl.lmax = all_blocks ? lcap : 1;
        // flag the blocks that may use vector lanes: all of them under the policy, else (unless disabled) the blocks
        // made only of split-row pieces (inexact anyway; a 16 M-nonzero row is thousands of one-piece blocks)
        auto dest_of = [&](int v) -> int64_t {
            if (in.vdest.empty()) return v;
            return (W > 0) ? (in.vdest[v] >> 1) : in.vdest[v];
        };
        bool any_flag = false;
        for (int2 &bk : in.blk) {
            bool ok = all_blocks;
            if (!ok && forced >= 0 && !in.long_rows.empty() && bk.y - bk.x < ng) {
                ok = true;
                for (int v = bk.x; v < bk.y && ok; ++v) ok = dest_of(v) < 0;
            }
            if (ok) bk.y |= BLK_VL_FLAG, any_flag = true;
        }
        if (any_flag && pl.lmax <= 1) pl.lmax = lcap;
        d.exact.assign((size_t)h->m, 1);
        for (const int4 &lr : in.long_rows) d.exact[(size_t)lr.x] = 0;
        if (pl.lmax > 1) {
            for (const int2 &bk : in.blk) {
                if (!(bk.y & BLK_VL_FLAG)) continue;
                const int e = bk.y & BLK_ROWS_MASK, nrows = e - bk.x;
                if (nrows >= ng) continue;
                int L = 1;
                while (2 * L <= ng / nrows) L *= 2;
                if (std::min(L, pl.lmax) <= 1) continue;
                for (int v = bk.x; v < e; ++v) {
                    const int64_t dd = dest_of(v);
                    if (dd >= 0) d.exact[(size_t)dd] = 0;
                }
            }
        }
        pl.exact_rows = 0;
        for (uint8_t e : d.exact) pl.exact_rows += e;
        // paired short rows: two rows of <= U/2 nonzeros share a gather round trip, the wave's groups
        // still in step.  No column windows, row groups of >= 2 lanes (one-lane groups hold 1-2 rows of a block);
        // blocks that take vector lanes keep their loop.  SPMM_HIP_PAIR=-1 off, 1 forced.
        const int env_pair = env_int("SPMM_HIP_PAIR", 0);
        const bool pair_ok = W == 0 && g >= 2 && nnz_rows > 0 && pl.cap <= CAP;
        if (pair_ok && env_pair > 0)
            pl.pair = 1;
        else if (pair_ok && env_pair == 0 && h->vsize == 8 && g <= PAIR_MAX_G && h->nnz >= PAIR_MIN_NNZ &&
                 mean_vrow <= PAIR_MAX_ROW && rows_per_block >= 2.0 * ng) {
            if (int st = load_cols()) return st;
            pl.pair_reuse = tile_reuse_sample(h->h_row_ptr.data(), hcol, h->m, h->ncols, INT32_MAX, PAIR_WINDOW_ROWS);
            if (pl.pair_reuse >= PAIR_MIN_REUSE) pl.pair = 1;
        }
    }
    // fused combine: split rows summed by the block that stores their last piece, so no combine
    // launch.  Needs one launch per panel (no column windows), partials below 4 GiB (32-bit buffer offsets) and each
    // split row's pieces in consecutive virtual rows with consecutive slots (what inspect() builds; checked here).
    // SPMM_HIP_FUSE=0 keeps the separate spmm_combine_kernel.
    {
        std::vector<int32_t> &slot_lr = d.slot_lr;
        const int nslots = in.nslots;
        bool fuse = nslots > 0 && W == 0 && !pl.ygrid && env_int("SPMM_HIP_FUSE", 1) != 0 &&
                    (uint64_t)nslots * (uint64_t)k * h->vsize < (1ULL << 32);
        if (fuse) {
            slot_lr.assign((size_t)nslots, -1);
            std::vector<int64_t> slot_v((size_t)nslots, -1);
            for (size_t v = 0; v < in.vdest.size(); ++v)
                if (in.vdest[v] < 0) slot_v[(size_t)(-in.vdest[v] - 1)] = (int64_t)v;
            for (size_t li = 0; li < in.long_rows.size() && fuse; ++li) {
                const int4 lr = in.long_rows[li];
                for (int q = 0; q < lr.z && fuse; ++q) {
                    const int sl = lr.y + q;
                    fuse = sl < nslots && slot_v[(size_t)sl] >= 0 && slot_lr[(size_t)sl] < 0 &&
                           (q == 0 || slot_v[(size_t)sl] == slot_v[(size_t)sl - 1] + 1);
                    if (fuse) slot_lr[(size_t)sl] = (int32_t)li;
                }
            }
            for (int32_t x : slot_lr) fuse = fuse && x >= 0;
        }
        if (fuse) {
            for (int2 &bk : in.blk) {
                const int e = bk.y & BLK_ROWS_MASK;
                for (int v = bk.x; v < e; ++v)
                    if (in.vdest[(size_t)v] < 0) {
                        bk.y |= BLK_SPLIT_FLAG;
                        break;
                    }
            }
        }
        d.fuse = fuse;
        if (!fuse) slot_lr.clear();
    }
    return SPMM_HIP_OK;
}

// FNV-1a over the plan's decisions and tables (spmm_hip_debug_plan: two builds or two policies plan a matrix the
// same way exactly when their fingerprints agree)
uint64_t plan_fingerprint(const Draft &d) {
    uint64_t x = 1469598103934665603ULL;
    auto mix = [&](const void *p, size_t n) {
        const unsigned char *c = (const unsigned char *)p;
        for (size_t i = 0; i < n; ++i) x = (x ^ c[i]) * 1099511628211ULL;
    };
    const Plan &p = d.pl;
    const int64_t f[] = {p.k, p.kw, p.npanels, p.ygrid, p.seq_max, p.piece, p.cap, p.block_rows, p.win_cols, p.nwin, p.nseg,
                         p.xcd, p.lmax, p.exact_rows, p.ntile, p.tile_xcd, p.tile_wide, p.tile_mfma, p.tile_rows,
                         p.tile_nnz, p.tile_chunks, (int64_t)d.fuse, p.pair};
    mix(f, sizeof(f));
    mix(d.in.vrow_ptr.data(), d.in.vrow_ptr.size() * 4);
    mix(d.in.vdest.data(), d.in.vdest.size() * 4);
    mix(d.in.blk.data(), d.in.blk.size() * sizeof(int2));
    mix(d.tp.tiles.data(), d.tp.tiles.size() * sizeof(int4));
    mix(d.tp.chunks.data(), d.tp.chunks.size() * sizeof(int4));
    return x;
}

}  // namespace

extern "C" {

#ifdef SPMM_STAMPS
// Diagnostic build only: point the row kernel's per-block stamps at a device buffer of >= 4 * blocks int64 (nullptr
// turns them off).  Not in include/spmm_hip.h: the shipped library has no such symbol.
int spmm_hip_debug_row_stamps(void *d_buf) {
    long long *p = (long long *)d_buf;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_row_stamps), &p, sizeof(p)));
    return SPMM_HIP_OK;
}
#endif
const char *spmm_hip_version(void) { return "spmm-mi355x 0.2 (gfx950 virtual-row block kernel)"; }

const char *spmm_hip_strerror(int s) {
    switch (s) {
        case SPMM_HIP_OK: return "ok";
        case SPMM_HIP_ERR_ARG: return "invalid argument";
        case SPMM_HIP_ERR_NOMEM: return "out of memory";
        case SPMM_HIP_ERR_HIP: return "HIP runtime error";
        case SPMM_HIP_ERR_NODEVICE: return "no such HIP device";
        case SPMM_HIP_ERR_K: return "k mismatch";
        case SPMM_HIP_ERR_CSR: return "malformed CSR";
        case SPMM_HIP_ERR_OVERFLOW: return "size overflow";
        default: return "unknown status";
    }
}

const char *spmm_hip_last_error_detail(void) { return g_detail.c_str(); }

int spmm_hip_device_count(int *count) {
    if (!count) return fail(SPMM_HIP_ERR_ARG, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return SPMM_HIP_OK;
}

double spmm_hip_bytes_alg(int64_t m, int64_t ncols, int64_t nnz, int32_t k, int32_t dtype) {
    const double s = (dtype == SPMM_HIP_F32) ? 4.0 : 8.0;
    return 4.0 * (double)(m + 1) + (4.0 + s) * (double)nnz + s * (double)k * (double)ncols +
           s * (double)k * (double)m;
}

// loop_partitioner_balance_prefix_sums (lib/parallel_util.h:141-165) with binary_search
// (lib/macros/macrolib.h:471-524, default comparator / distance :440-448).
static int64_t bsearch_nearest(const int32_t *A, int64_t lo, int64_t hi, int64_t target) {
    int64_t s = lo, e = hi;
    if (target < A[s]) return s;
    if (target > A[e]) return e;
    for (;;) {
        const int64_t mid = (s + e) / 2;
        if (mid == s || mid == e) break;
        if (target > A[mid])
            s = mid;
        else
            e = mid;
    }
    if (target == A[s]) return s;
    if (target == A[e]) return e;
    const int64_t ds = target - A[s] < 0 ? A[s] - target : target - A[s];
    const int64_t de = target - A[e] < 0 ? A[e] - target : target - A[e];
    return ds < de ? s : e;
}

int spmm_hip_partition_rows(const int32_t *row_ptr, int64_t m, int64_t nnz, int64_t W, int64_t w, int64_t *start,
                            int64_t *end) {
    if (!row_ptr || !start || !end || m < 1 || W < 1 || w < 0 || w >= W)
        return fail(SPMM_HIP_ERR_ARG, "partition: bad arguments");
    const int64_t t0 = (nnz * w) / W, t1 = (nnz * (w + 1)) / W;
    *start = (w == 0) ? 0 : bsearch_nearest(row_ptr, 0, m - 1, t0);
    *end = (w == W - 1) ? m : bsearch_nearest(row_ptr, 0, m - 1, t1);
    return SPMM_HIP_OK;
}

int spmm_hip_create(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m, int64_t ncols,
                    int64_t nnz, int32_t k, int32_t dtype, int32_t device, spmm_hip_t **out) {
    if (!out) return fail(SPMM_HIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (m < 0 || ncols < 0 || nnz < 0 || k < 0) return fail(SPMM_HIP_ERR_ARG, "negative size");
    if (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32) return fail(SPMM_HIP_ERR_ARG, "dtype");
    if (!row_ptr || (nnz > 0 && (!col_idx || !values))) return fail(SPMM_HIP_ERR_ARG, "null CSR array");
    if (m >= INT32_MAX || ncols >= INT32_MAX || nnz >= INT32_MAX - 4096)
        return fail(SPMM_HIP_ERR_OVERFLOW, "m, ncols and nnz must fit int32 (reference INT_T = int32_t)");
    // validate the CSR (the reference trusts its input; we refuse malformed input instead of faulting the GPU)
    if (row_ptr[0] != 0 || row_ptr[m] != nnz) return fail(SPMM_HIP_ERR_CSR, "row_ptr[0] != 0 or row_ptr[m] != nnz");
    for (int64_t i = 0; i < m; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return fail(SPMM_HIP_ERR_CSR, "row_ptr not monotone at row " + std::to_string(i));
    for (int64_t j = 0; j < nnz; ++j)
        if (col_idx[j] < 0 || col_idx[j] >= ncols)
            return fail(SPMM_HIP_ERR_CSR, "col_idx out of range at nonzero " + std::to_string(j));

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SPMM_HIP_ERR_NODEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(SPMM_HIP_ERR_NODEVICE, "device index out of range");
    HIPCHK(hipSetDevice(device));

    spmm_hip_t *h = new spmm_hip_t();
    h->device = device;
    h->dtype = dtype;
    h->vsize = (dtype == SPMM_HIP_F64) ? 8 : 4;
    h->m = m;
    h->ncols = ncols;
    h->nnz = nnz;
    h->h_row_ptr.assign(row_ptr, row_ptr + m + 1);

    auto cleanup = [&](int st) {
        spmm_hip_destroy(h);
        return st;
    };
#define HIPCHK_C(expr)                                                                                   \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess) {                                                                          \
            int _s = (_e == hipErrorOutOfMemory) ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP;                 \
            fail(_s, std::string(#expr) + ": " + hipGetErrorString(_e));                                 \
            return cleanup(_s);                                                                          \
        }                                                                                                \
    } while (0)

    const size_t col_b = (size_t)nnz * 4 + PAD_BYTES, val_b = (size_t)nnz * h->vsize + PAD_BYTES;
    HIPCHK_C(hipMalloc(&h->d_col, col_b));
    HIPCHK_C(hipMalloc(&h->d_val, val_b));
    HIPCHK_C(hipMemset(h->d_col, 0, col_b));
    HIPCHK_C(hipMemset(h->d_val, 0, val_b));
    if (nnz > 0) {
        HIPCHK_C(hipMemcpy(h->d_col, col_idx, (size_t)nnz * 4, hipMemcpyHostToDevice));
        HIPCHK_C(hipMemcpy(h->d_val, values, (size_t)nnz * h->vsize, hipMemcpyHostToDevice));
    }
    h->a_bytes = (int64_t)(col_b + val_b);
    HIPCHK_C(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    for (auto &e : h->ev) HIPCHK_C(hipEventCreate(&e));
    h->rec_events = env_int("SPMM_HIP_EVENTS", 0) != 0;
#undef HIPCHK_C
    if (k > 0) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return cleanup(st);
    }
    *out = h;
    return SPMM_HIP_OK;
}

int spmm_hip_plan(spmm_hip_t *h, int32_t k) {
    if (!h || k < 1) return fail(SPMM_HIP_ERR_ARG, "plan: bad handle or k < 1");
    if (h->plan.k == k) return SPMM_HIP_OK;
    if (h->multi) return multi_plan(h, k);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    free_plan(h);
    Draft d;
    if (int st = draft_plan(h, k, nullptr, false, d)) return st;
    const Plan &pl = d.pl;
    TilePlan &tp = d.tp;
    const bool tiles = d.tiles;
    Inspection &in = d.in;
    const int64_t W = d.W;
    const std::vector<int32_t> &slot_lr = d.slot_lr;
    const int64_t srow_t = (int64_t)pl.kw * (int64_t)h->vsize;
    h->nv = (int64_t)in.vrow_ptr.size() - 1;
    h->nblk = (int)in.blk.size();
    h->nlong = (int)in.long_rows.size();
    h->nslots = in.nslots;
    h->exact.swap(d.exact);
    h->fuse = d.fuse;
    h->plan = pl;
    h->win_blk = in.win_blk;
    h->win_v = in.win_v;
    std::vector<int32_t> hcol;     // the tile / window copies below re-read the columns
    if (W > 0) {
        hcol.resize((size_t)h->nnz);
        HIPCHK(hipMemcpy(hcol.data(), h->d_col, (size_t)h->nnz * 4, hipMemcpyDeviceToHost));
    }

    auto alloc_copy = [&](void **dst, const void *src, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(dst, std::max<size_t>(bytes, 4));
        if (e == hipSuccess && bytes > 0) e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
        return e;
    };
    hipError_t e = alloc_copy((void **)&h->d_vrow_ptr, in.vrow_ptr.data(), in.vrow_ptr.size() * 4);
    {   // device block table carries the block's nonzero range too: one 16-B load instead of two dependent ones
        std::vector<int4> blk4(in.blk.size());
        for (size_t b = 0; b < in.blk.size(); ++b) {
            const int2 bk = in.blk[b];
            blk4[b] = make_int4(bk.x, bk.y, in.vrow_ptr[(size_t)bk.x], in.vrow_ptr[(size_t)(bk.y & BLK_ROWS_MASK)]);
        }
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_blk, blk4.data(), blk4.size() * sizeof(int4));
    }
    if (e == hipSuccess && !in.vdest.empty()) e = alloc_copy((void **)&h->d_vdest, in.vdest.data(), in.vdest.size() * 4);
    if (e == hipSuccess && h->nlong > 0)
        e = alloc_copy((void **)&h->d_long_rows, in.long_rows.data(), in.long_rows.size() * sizeof(int4));
    if (e == hipSuccess && h->fuse) {
        e = alloc_copy((void **)&h->d_slot_lr, slot_lr.data(), slot_lr.size() * 4);
        if (e == hipSuccess) e = hipMalloc((void **)&h->d_lr_cnt, (size_t)h->nlong * 4);
        if (e == hipSuccess) e = hipMemset(h->d_lr_cnt, 0, (size_t)h->nlong * 4);
    }
    h->insp_bytes = (in.vrow_ptr.size() + in.vdest.size()) * 4 + in.blk.size() * sizeof(int4) +
                    in.long_rows.size() * sizeof(int4);
    h->b_bytes = (size_t)std::max<int64_t>(h->ncols, 1) * k * h->vsize;
    h->c_bytes = (size_t)std::max<int64_t>(h->m, 1) * k * h->vsize;
    // the handle's own B / staging / C buffers are allocated at first use (ensure_buffers): a caller that keeps B
    // and C in its own HBM (spmm_hip_run_device with a row-major B) never pays for them
    if (e == hipSuccess && h->nslots > 0) e = hipMalloc(&h->d_part, (size_t)h->nslots * k * h->vsize);
    if (e == hipSuccess && W > 0) {
        // window-major copies of col_idx / values (same padding as the originals)
        const size_t nz = in.perm.size();
        std::vector<char> hval((size_t)h->nnz * h->vsize), wval(nz * h->vsize + PAD_BYTES, 0);
        std::vector<int32_t> wcol(nz + PAD_BYTES / 4, 0);
        e = hipMemcpy(hval.data(), h->d_val, hval.size(), hipMemcpyDeviceToHost);
        for (size_t q = 0; q < nz; ++q) {
            const int64_t j = in.perm[q];
            wcol[q] = hcol[(size_t)j];
            std::memcpy(&wval[q * h->vsize], &hval[(size_t)j * h->vsize], h->vsize);
        }
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_wcol, wcol.data(), wcol.size() * 4);
        if (e == hipSuccess) e = alloc_copy(&h->d_wval, wval.data(), wval.size());
        std::vector<int32_t> wp(in.perm.begin(), in.perm.end());
        h->nwperm = (int64_t)wp.size();
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_wperm, wp.data(), wp.size() * 4);
        h->insp_bytes += wcol.size() * 4 + wval.size();
    }
    if (e == hipSuccess && tiles && pl.tile_mfma) {
        std::vector<char> hval((size_t)h->nnz * h->vsize);
        e = hipMemcpy(hval.data(), h->d_val, hval.size(), hipMemcpyDeviceToHost);
        const size_t nz = tp.perm.size();
        std::vector<char> tval(nz * h->vsize + PAD_BYTES, 0);
        for (size_t q = 0; q < nz; ++q)
            if (tp.perm[q] >= 0) std::memcpy(&tval[q * h->vsize], &hval[(size_t)tp.perm[q] * h->vsize], h->vsize);
        {
            // matrix-core tables: each entry's panel cell (row in tile * PST + chunk column; padding -> the trash
            // cell) and each chunk's union columns in [g][k step] order, 48 slots, padded with a valid row
            const int64_t nch = (int64_t)tp.chunks.size() - 1;
            std::vector<uint16_t> cell(nz + PAD_BYTES / 2, (uint16_t)MFMA_TRASH);
            std::vector<int32_t> tcolT((size_t)nch * MFMA_UC + PAD_BYTES / 4, 0);
            for (const int4 &t : tp.tiles)
                for (int ci = t.z; ci < t.z + t.w; ++ci) {
                    const int4 ch = tp.chunks[(size_t)ci];
                    for (int q = 0; q < t.y; ++q)
                        for (int p = tp.tseg[(size_t)ch.w + q]; p < tp.tseg[(size_t)ch.w + q + 1]; ++p) {
                            const uint16_t lc = tp.tlidx[(size_t)ch.z + p];
                            if (lc != TILE_PAD_LIDX) cell[(size_t)ch.z + p] = (uint16_t)(q * MFMA_PST + lc);
                        }
                    for (int u = 0; u < MFMA_UC; ++u)
                        tcolT[(size_t)ci * MFMA_UC + (u % 4) * MFMA_KS + u / 4] = tp.tcol[(size_t)ch.x + std::min(u, ch.y - 1)];
                }
            // A's exact range (spmm_mfma.hpp): mflag[0] = some tile value outside it; mflag[1] is B's, per launch
            int mflag[2] = {0, 0};
            for (size_t q = 0; q < nz && !mflag[0]; ++q) {
                if (tp.perm[q] < 0) continue;
                double v;
                if (h->vsize == 8) std::memcpy(&v, &tval[q * 8], 8);
                else { float f; std::memcpy(&f, &tval[q * 4], 4); v = f; }
                int ex = 0;
                (void)std::frexp(v, &ex);
                const int lo = h->vsize == 8 ? MfmaT<double>::MIN_EXP : MfmaT<float>::MIN_EXP;
                const int hi = h->vsize == 8 ? MfmaT<double>::MAX_EXP : MfmaT<float>::MAX_EXP;
                mflag[0] = !std::isfinite(v) || (v != 0.0 && (ex < lo || ex > hi));
            }
            if (e == hipSuccess) e = alloc_copy((void **)&h->d_mflag, mflag, sizeof(mflag));
            if (e == hipSuccess) e = alloc_copy((void **)&h->d_tiles, tp.tiles.data(), tp.tiles.size() * sizeof(int4));
            if (e == hipSuccess) e = alloc_copy((void **)&h->d_tchunk, tp.chunks.data(), tp.chunks.size() * sizeof(int4));
            if (e == hipSuccess) e = alloc_copy((void **)&h->d_tcol, tcolT.data(), tcolT.size() * 4);
            if (e == hipSuccess) e = alloc_copy((void **)&h->d_tlidx, cell.data(), cell.size() * 2);
            // the values (and the value-update gather map) in the kernel's per-chunk order (spmm_mfma.hpp: 16-byte
            // entry loads); the cells stay in entry order
            std::vector<int32_t> tpm(tp.perm.size(), -1);
            {
                std::vector<char> tvp(tval.size(), 0);
                for (size_t ci = 0; ci + 1 < tp.chunks.size(); ++ci) {
                    const int z = tp.chunks[ci].z, ne = tp.chunks[ci + 1].z - z;
                    for (int q = 0; q < ne; ++q) {
                        const int pos = h->vsize == 8 ? mfma_val_pos<double>(q, ne / 8) : mfma_val_pos<float>(q, ne / 8);
                        std::memcpy(&tvp[(size_t)(z + pos) * h->vsize], &tval[(size_t)(z + q) * h->vsize], h->vsize);
                        tpm[(size_t)(z + pos)] = (int32_t)tp.perm[(size_t)(z + q)];
                    }
                }
                tval.swap(tvp);
            }
            if (e == hipSuccess) e = alloc_copy(&h->d_tval, tval.data(), tval.size());
            h->ntperm = (int64_t)tpm.size();
            if (e == hipSuccess) e = alloc_copy((void **)&h->d_tperm, tpm.data(), tpm.size() * 4);
            h->insp_bytes += tp.tiles.size() * sizeof(int4) + tp.chunks.size() * sizeof(int4) + tcolT.size() * 4 +
                             cell.size() * 2 + tval.size() + tpm.size() * 4;
        }
    }
    if (e == hipSuccess && tiles && !pl.tile_mfma) {
        // chunk-major copies of the tile rows' values and their chunk-local column indices (+ 64 B of padding).
        // A padding entry is (value -0, the zero B row): fma(-0, +0, acc) == acc for every acc, -0 included (a +0
        // value would turn a -0 chain, which the reference can reach through underflow, into +0)
        std::vector<char> hval((size_t)h->nnz * h->vsize);
        e = hipMemcpy(hval.data(), h->d_val, hval.size(), hipMemcpyDeviceToHost);
        const size_t nz = tp.perm.size();
        std::vector<char> tval(nz * h->vsize + PAD_BYTES, 0);
        const double mz64 = -0.0;
        const float mz32 = -0.0f;
        for (size_t q = 0; q < nz; ++q) {
            if (tp.perm[q] >= 0)
                std::memcpy(&tval[q * h->vsize], &hval[(size_t)tp.perm[q] * h->vsize], h->vsize);
            else
                std::memcpy(&tval[q * h->vsize], h->vsize == 8 ? (const void *)&mz64 : (const void *)&mz32, h->vsize);
        }
        // chunk-local column -> byte offset of its row in the staged B image (padding: the zero row after the image)
        for (uint16_t &l : tp.tlidx) l = (l == TILE_PAD_LIDX) ? (uint16_t)TILE_UCB : (uint16_t)(l * srow_t);
        tp.tlidx.resize(nz + PAD_BYTES / 2, 0);
        tp.tseg.resize(tp.tseg.size() + PAD_BYTES / 2, 0);
        tp.tcol.resize(tp.tcol.size() + PAD_BYTES / 4, 0);
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_tiles, tp.tiles.data(), tp.tiles.size() * sizeof(int4));
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_tchunk, tp.chunks.data(), tp.chunks.size() * sizeof(int4));
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_tcol, tp.tcol.data(), tp.tcol.size() * 4);
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_tseg, tp.tseg.data(), tp.tseg.size() * 2);
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_tlidx, tp.tlidx.data(), tp.tlidx.size() * 2);
        if (e == hipSuccess) e = alloc_copy(&h->d_tval, tval.data(), tval.size());
        std::vector<int32_t> tpm(tp.perm.begin(), tp.perm.end());
        h->ntperm = (int64_t)tpm.size();
        if (e == hipSuccess) e = alloc_copy((void **)&h->d_tperm, tpm.data(), tpm.size() * 4);
        if (e == hipSuccess && env_int("SPMM_HIP_TILE_STAMPS", 0)) {
            e = hipMalloc((void **)&h->d_tstamps, tp.tiles.size() * 4 * sizeof(long long));
            if (e == hipSuccess) e = hipMemset(h->d_tstamps, 0, tp.tiles.size() * 4 * sizeof(long long));
        }
        h->insp_bytes += tp.tiles.size() * sizeof(int4) + tp.chunks.size() * sizeof(int4) + tp.tcol.size() * 4 +
                         tp.tseg.size() * 2 + tp.tlidx.size() * 2 + tval.size();
    }
    // the side stream of matrix-core plans (created here, never inside a run: runs may be graph-captured)
    if (e == hipSuccess && h->plan.tile_mfma && !h->side) {
        e = hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        free_plan(h);
        return fail(e == hipErrorOutOfMemory ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP,
                    std::string("plan alloc: ") + hipGetErrorString(e));
    }
    return SPMM_HIP_OK;
}

int spmm_hip_run_device(spmm_hip_t *h, const void *d_b, int32_t b_layout, void *d_c, int32_t k, void *stream) {
    if (!h || !d_b || !d_c || k < 1) return fail(SPMM_HIP_ERR_ARG, "run_device: bad arguments");
    if (b_layout != SPMM_HIP_B_COL_MAJOR && b_layout != SPMM_HIP_B_ROW_MAJOR)
        return fail(SPMM_HIP_ERR_ARG, "run_device: b_layout");
    if (h->plan.k != k) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return st;
    }
    if (((uintptr_t)d_b | (uintptr_t)d_c) % 16 != 0)
        return fail(SPMM_HIP_ERR_ARG, "run_device: device buffers must be 16-byte aligned");
    if (h->multi) return multi_run_device(h, d_b, b_layout, d_c, k, (hipStream_t)stream);
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const void *B = d_b;
    const bool ev = h->rec_events;
    h->have_transpose = false;
    if (b_layout == SPMM_HIP_B_COL_MAJOR) {
        if (int st = ensure_buffers(h, true, false, false)) return st;
        // h->d_b is about to hold THIS B: a later spmm_hip_run(x) must not skip its upload on the strength of
        // SPMM_HIP_ASSUME_X_UNCHANGED (its cached x is no longer what d_b holds)
        h->last_x = nullptr;
        if (ev) HIPCHK(hipEventRecord(h->ev[2], s));
        int st = launch_transpose(h, d_b, h->d_b, k, s);
        if (st != SPMM_HIP_OK) return st;
        if (ev) HIPCHK(hipEventRecord(h->ev[3], s));
        B = h->d_b;
        h->have_transpose = ev;
    }
    if (ev) HIPCHK(hipEventRecord(h->ev[0], s));
    if (h->m > 0) {
        int st = launch_spmm(h, B, d_c, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    if (ev) HIPCHK(hipEventRecord(h->ev[1], s));
    h->have_times = ev;
    h->have_copies = false;
    return SPMM_HIP_OK;
}

}  // extern "C"

namespace {
// Side streams and fork/join events of spmm_hip_run_device_batch, per device, created on first use and kept.
struct BatchPool {
    std::vector<hipStream_t> side;
    std::vector<hipEvent_t> join;
    hipEvent_t fork = nullptr;
};
std::mutex g_batch_mu;
std::map<int, BatchPool> g_batch_pools;
}  // namespace

extern "C" {

int spmm_hip_run_device_batch(int32_t count, spmm_hip_t *const *hs, const void *const *d_b, const int32_t *b_layout,
                              void *const *d_c, const int32_t *k, void *stream) {
    if (count < 1 || !hs || !d_b || !b_layout || !d_c || !k) return fail(SPMM_HIP_ERR_ARG, "run_device_batch: bad arguments");
    for (int i = 0; i < count; ++i) {
        if (!hs[i]) return fail(SPMM_HIP_ERR_ARG, "run_device_batch: null handle");
        if (hs[i]->multi) return fail(SPMM_HIP_ERR_ARG, "run_device_batch: multi-GPU handles fan out on their own");
        if (hs[i]->device != hs[0]->device) return fail(SPMM_HIP_ERR_ARG, "run_device_batch: handles on different devices");
        for (int j = 0; j < i; ++j)
            if (hs[j] == hs[i]) return fail(SPMM_HIP_ERR_ARG, "run_device_batch: a handle appears twice");
    }
    if (count == 1) return spmm_hip_run_device(hs[0], d_b[0], b_layout[0], d_c[0], k[0], stream);
    // plan (host work, may allocate) before the fork, so nothing below allocates inside a graph capture
    for (int i = 0; i < count; ++i)
        if (hs[i]->plan.k != k[i]) {
            int st = spmm_hip_plan(hs[i], k[i]);
            if (st != SPMM_HIP_OK) return st;
        }
    std::lock_guard<std::mutex> lock(g_batch_mu);
    const int dev = hs[0]->device;
    HIPCHK(hipSetDevice(dev));
    BatchPool &pool = g_batch_pools[dev];
    if (!pool.fork) HIPCHK(hipEventCreateWithFlags(&pool.fork, hipEventDisableTiming));
    while ((int)pool.side.size() < count - 1) {
        hipStream_t st;
        hipEvent_t ev;
        HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        pool.side.push_back(st);
        pool.join.push_back(ev);
    }
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipEventRecord(pool.fork, s));
    // From here on every side stream that joined the fork is joined back into `stream` even when a run fails, so
    // a graph capture on `stream` stays well formed and the first error is what the caller sees.
    int first = SPMM_HIP_OK;
    std::string first_detail;
    auto keep = [&](int st) {
        if (st != SPMM_HIP_OK && first == SPMM_HIP_OK) first = st, first_detail = g_detail;
    };
    std::vector<char> forked((size_t)count, 0);
    for (int i = 1; i < count && first == SPMM_HIP_OK; ++i) {
        hipError_t e = hipStreamWaitEvent(pool.side[i - 1], pool.fork, 0);
        if (e != hipSuccess) {
            keep(fail(SPMM_HIP_ERR_HIP, std::string("hipStreamWaitEvent(fork): ") + hipGetErrorString(e)));
            break;
        }
        forked[(size_t)i] = 1;
        keep(spmm_hip_run_device(hs[i], d_b[i], b_layout[i], d_c[i], k[i], pool.side[i - 1]));
    }
    if (first == SPMM_HIP_OK) keep(spmm_hip_run_device(hs[0], d_b[0], b_layout[0], d_c[0], k[0], s));
    for (int i = 1; i < count; ++i) {
        if (!forked[(size_t)i]) continue;
        hipError_t e = hipEventRecord(pool.join[i - 1], pool.side[i - 1]);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, pool.join[i - 1], 0);
        if (e != hipSuccess) keep(fail(SPMM_HIP_ERR_HIP, std::string("batch join: ") + hipGetErrorString(e)));
    }
    if (first != SPMM_HIP_OK) g_detail = first_detail;
    return first;
}

}  // extern "C"

namespace {
// dst[q] = perm[q] >= 0 ? src[perm[q]] : 0 (the window-major / tile chunk-major copies of A's values)
// flag != nullptr (matrix-core tiles): also sets *flag when a gathered value lies outside the exact range
// (spmm_mfma.hpp, mflag[0])
template <typename T>
__global__ __launch_bounds__(WG) void gather_values_kernel(const T *__restrict__ src, const int32_t *__restrict__ perm,
                                                           T *__restrict__ dst, int64_t n, int *__restrict__ flag) {
    const int64_t q = (int64_t)blockIdx.x * WG + threadIdx.x;
    bool bad = false;
    if (q < n) {
        const int32_t j = perm[q];
        const T v = j >= 0 ? src[j] : T(-0.0);    // padding: -0 (LDS tiles: fma(-0, +0, acc) == acc, -0 kept)
        dst[q] = v;
        if (flag) {
            const int ex = MfmaT<T>::fexp(v);
            bad = !__builtin_isfinite(v) || (v != T(0) && (ex < MfmaT<T>::MIN_EXP || ex > MfmaT<T>::MAX_EXP));
        }
    }
    if (flag && __builtin_amdgcn_ballot_w64(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

int update_values(spmm_hip_t *h, const void *vals, hipMemcpyKind kind, hipStream_t s) {
    if (h->nnz == 0) return SPMM_HIP_OK;
    HIPCHK(hipMemcpyAsync(h->d_val, vals, (size_t)h->nnz * h->vsize, kind, s));
    auto gather = [&](const int32_t *perm, void *dst, int64_t n, int *flag) -> int {
        if (!perm || n == 0) return SPMM_HIP_OK;
        const unsigned nb = (unsigned)((n + WG - 1) / WG);
        if (flag) HIPCHK(hipMemsetAsync(flag, 0, sizeof(int), s));
        if (h->dtype == SPMM_HIP_F64)
            gather_values_kernel<double><<<nb, WG, 0, s>>>((const double *)h->d_val, perm, (double *)dst, n, flag);
        else
            gather_values_kernel<float><<<nb, WG, 0, s>>>((const float *)h->d_val, perm, (float *)dst, n, flag);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? SPMM_HIP_OK : fail(SPMM_HIP_ERR_HIP, std::string("gather launch: ") + hipGetErrorString(e));
    };
    if (int st = gather(h->d_wperm, h->d_wval, h->nwperm, nullptr)) return st;
    if (int st = gather(h->d_tperm, h->d_tval, h->ntperm, h->plan.tile_mfma ? h->d_mflag : nullptr)) return st;
    return SPMM_HIP_OK;
}
}  // namespace

extern "C" {

int spmm_hip_update_values_device(spmm_hip_t *h, const void *d_vals, void *stream) {
    if (!h || (!d_vals && h->nnz > 0)) return fail(SPMM_HIP_ERR_ARG, "update_values_device: bad arguments");
    if (h->multi) return multi_update_values(h, d_vals, true, (hipStream_t)stream);
    HIPCHK(hipSetDevice(h->device));
    return update_values(h, d_vals, hipMemcpyDeviceToDevice, (hipStream_t)stream);
}

int spmm_hip_update_values(spmm_hip_t *h, const void *vals) {
    if (!h || (!vals && h->nnz > 0)) return fail(SPMM_HIP_ERR_ARG, "update_values: bad arguments");
    if (h->multi) return multi_update_values(h, vals, false, nullptr);
    HIPCHK(hipSetDevice(h->device));
    int st = update_values(h, vals, hipMemcpyHostToDevice, h->stream);
    if (st != SPMM_HIP_OK) return st;
    HIPCHK(hipStreamSynchronize(h->stream));
    return SPMM_HIP_OK;
}

// Host buffers, B ROW-major (x[col*k + n], the layout MKL's csrmm takes in the reference pipeline plugin,
// pipeline_code_bench/sddmm_taco_naive.cpp:219-249): upload straight into the engine's B, no transpose.
int spmm_hip_run_rowmajor(spmm_hip_t *h, const void *x, void *y, int32_t k) {
    if (!h || k < 1 || (!x && h->ncols > 0) || (!y && h->m > 0)) return fail(SPMM_HIP_ERR_ARG, "run_rowmajor: bad arguments");
    if (h->multi) return multi_run_host(h, x, y, k, true);
    if (h->plan.k != k) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return st;
    }
    if (int st = ensure_buffers(h, true, false, true)) return st;
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    h->last_x = nullptr;
    HIPCHK(hipEventRecord(h->ev[4], s));
    if (h->ncols > 0) HIPCHK(hipMemcpyAsync(h->d_b, x, (size_t)h->ncols * k * h->vsize, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(h->ev[5], s));
    HIPCHK(hipEventRecord(h->ev[0], s));
    if (h->m > 0) {
        int st = launch_spmm(h, h->d_b, h->d_c, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipEventRecord(h->ev[1], s));
    if (h->m > 0) HIPCHK(hipMemcpyAsync(y, h->d_c, (size_t)h->m * k * h->vsize, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(h->ev[6], s));
    HIPCHK(hipStreamSynchronize(s));
    h->have_times = h->have_copies = true;
    h->have_transpose = false;
    return SPMM_HIP_OK;
}

int spmm_hip_run(spmm_hip_t *h, const void *x, void *y, int32_t k) {
    if (!h || k < 1 || (!x && h->ncols > 0) || (!y && h->m > 0)) return fail(SPMM_HIP_ERR_ARG, "run: bad arguments");
    if (h->multi) return multi_run_host(h, x, y, k, false);
    if (h->plan.k != k) {
        int st = spmm_hip_plan(h, k);
        if (st != SPMM_HIP_OK) return st;
    }
    if (int st = ensure_buffers(h, true, true, true)) return st;
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const char *env = getenv("SPMM_HIP_ASSUME_X_UNCHANGED");
    const bool reuse = env && env[0] == '1' && x == h->last_x;
    HIPCHK(hipEventRecord(h->ev[4], s));
    if (!reuse && h->ncols > 0)
        HIPCHK(hipMemcpyAsync(h->d_xcol, x, (size_t)h->ncols * k * h->vsize, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(h->ev[5], s));
    HIPCHK(hipEventRecord(h->ev[2], s));
    if (!reuse) {
        int st = launch_transpose(h, h->d_xcol, h->d_b, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipEventRecord(h->ev[3], s));
    HIPCHK(hipEventRecord(h->ev[0], s));
    if (h->m > 0) {
        int st = launch_spmm(h, h->d_b, h->d_c, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    HIPCHK(hipEventRecord(h->ev[1], s));
    if (h->m > 0) HIPCHK(hipMemcpyAsync(y, h->d_c, (size_t)h->m * k * h->vsize, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(h->ev[6], s));
    HIPCHK(hipStreamSynchronize(s));
    h->last_x = x;
    h->have_times = h->have_transpose = h->have_copies = true;
    return SPMM_HIP_OK;
}

int spmm_hip_set_timing(spmm_hip_t *h, int32_t on) {
    if (!h) return fail(SPMM_HIP_ERR_ARG, "set_timing: handle is NULL");
    h->rec_events = on != 0;
    return SPMM_HIP_OK;
}

int spmm_hip_last_times(spmm_hip_t *h, double *out_ms) {
    if (!h || !out_ms) return fail(SPMM_HIP_ERR_ARG, "last_times: bad arguments");
    if (h->multi) return multi_last_times(h, out_ms);
    for (int i = 0; i < 4; ++i) out_ms[i] = 0.0;
    if (!h->have_times) return SPMM_HIP_OK;
    float ms = 0.f;
    HIPCHK(hipEventSynchronize(h->ev[1]));
    HIPCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    out_ms[0] = ms;
    if (h->have_transpose) {
        HIPCHK(hipEventElapsedTime(&ms, h->ev[2], h->ev[3]));
        out_ms[1] = ms;
    }
    if (h->have_copies) {
        HIPCHK(hipEventSynchronize(h->ev[6]));
        HIPCHK(hipEventElapsedTime(&ms, h->ev[4], h->ev[5]));
        out_ms[2] = ms;
        HIPCHK(hipEventElapsedTime(&ms, h->ev[1], h->ev[6]));
        out_ms[3] = ms;
    }
    return SPMM_HIP_OK;
}

int spmm_hip_stats_labels(char *buf, long buf_n) {
    if (!buf || buf_n <= 0) return fail(SPMM_HIP_ERR_ARG, "stats_labels: buffer");
    int n = snprintf(buf, (size_t)buf_n,
                     ",kernel_ms,transpose_ms,h2d_ms,d2h_ms,bytes_alg,hbm_gbs_alg,roofline_frac,blocks,split_rows,"
                     "seq_max,panels,windows,device,ngpus");
    return (int)std::min<long>(n, buf_n - 1);
}

int spmm_hip_stats(spmm_hip_t *h, char *buf, long buf_n) {
    if (!h || !buf || buf_n <= 0) return fail(SPMM_HIP_ERR_ARG, "stats: bad arguments");
    double t[4];
    int st = spmm_hip_last_times(h, t);
    if (st != SPMM_HIP_OK) return st;
    const int k = h->plan.k > 0 ? h->plan.k : 0;
    const double bytes = spmm_hip_bytes_alg(h->m, h->ncols, h->nnz, k, h->dtype);
    const double gbs = t[0] > 0 ? bytes / (t[0] * 1e-3) / 1e9 : 0.0;
    int64_t inf[SPMM_HIP_INFO_SLOTS];
    spmm_hip_info(h, inf);
    int32_t ng = 1;
    spmm_hip_ngpus(h, &ng, nullptr);
    // roofline_frac against ONE GPU's 8 TB/s (a multi-GPU handle's rate is the sum over its ngpus GPUs)
    int n = snprintf(buf, (size_t)buf_n, ",%.6f,%.6f,%.6f,%.6f,%.0f,%.2f,%.4f,%lld,%lld,%d,%d,%d,%d,%d", t[0], t[1],
                     t[2], t[3], bytes, gbs, gbs / 8000.0 / ng, (long long)inf[5], (long long)inf[6], h->plan.seq_max,
                     h->plan.npanels, h->plan.nwin, h->device, ng);
    return (int)std::min<long>(n, buf_n - 1);
}

int spmm_hip_info(const spmm_hip_t *h, int64_t *out) {
    if (!h || !out) return fail(SPMM_HIP_ERR_ARG, "info: bad arguments");
    out[0] = h->m;
    out[1] = h->ncols;
    out[2] = h->nnz;
    out[3] = h->plan.k;
    out[4] = h->dtype;
    out[5] = h->nblk;
    out[6] = h->nlong;
    out[7] = h->a_bytes + (int64_t)h->insp_bytes + (h->d_b ? (int64_t)h->b_bytes : 0) +
             (h->d_xcol ? (int64_t)h->b_bytes : 0) + (h->d_c ? (int64_t)h->c_bytes : 0) +
             (int64_t)h->nslots * std::max(h->plan.k, 0) * (int64_t)h->vsize;
    out[8] = h->plan.seq_max;
    out[9] = h->plan.cap;
    out[10] = h->plan.kw;
    out[11] = h->plan.npanels;
    out[12] = h->plan.nwin;
    out[13] = h->plan.win_cols;
    out[14] = h->plan.nseg;
    out[15] = h->plan.xcd;
    out[16] = h->plan.lmax;
    out[17] = h->plan.exact_rows;
    out[18] = h->fuse ? 1 : 0;
    out[19] = h->plan.ntile;
    if (h->multi) multi_info(h, out);     // blocks, split rows, device bytes, fuse: summed over the shards
    return SPMM_HIP_OK;
}

// Measurement only (SPMM_HIP_TILE_STAMPS=1 at plan time): per tile {start, end, wait, compute} s_memtime stamps of
// the last tile launch.  Not in the public header.
int spmm_hip_tile_stamps(spmm_hip_t *h, int64_t *out, int64_t n) {
    if (!h || !out || !h->d_tstamps) return fail(SPMM_HIP_ERR_ARG, "tile_stamps: not enabled");
    const int64_t cnt = std::min<int64_t>(n, (int64_t)h->plan.ntile * 4);
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, h->d_tstamps, (size_t)cnt * 8, hipMemcpyDeviceToHost));
    return SPMM_HIP_OK;
}

int spmm_hip_tile_info(const spmm_hip_t *h, int64_t *out) {
    if (!h || !out) return fail(SPMM_HIP_ERR_ARG, "tile_info: bad arguments");
    out[0] = h->plan.ntile;
    out[1] = h->plan.tile_rows;
    out[2] = h->plan.tile_nnz;
    out[3] = h->plan.tile_chunks;
    out[4] = (int64_t)(h->plan.tile_reuse * 1000.0 + 0.5);
    out[5] = h->plan.tile_xcd;
    out[6] = h->plan.tile_wide;
    return SPMM_HIP_OK;
}

int spmm_hip_tile_mode(const spmm_hip_t *h) {
    if (!h) return fail(SPMM_HIP_ERR_ARG, "tile_mode: bad handle");
    if (h->multi) return multi_tile_mode(h);
    return h->plan.ntile == 0 ? 0 : h->plan.tile_mfma ? 2 : 1;
}

int spmm_hip_exact_rows(const spmm_hip_t *h, uint8_t *mask) {
    if (!h || !mask || h->plan.k < 1) return fail(SPMM_HIP_ERR_ARG, "exact_rows: handle not planned");
    if (h->m > 0) std::memcpy(mask, h->exact.data(), (size_t)h->m);
    return SPMM_HIP_OK;
}

int spmm_hip_device_ptrs(spmm_hip_t *h, void **d_b_rowmajor, void **d_c) {
    if (!h || h->plan.k < 1) return fail(SPMM_HIP_ERR_ARG, "device_ptrs: handle not planned");
    if (h->multi) return fail(SPMM_HIP_ERR_ARG, "device_ptrs: a multi-GPU handle has no single C (spmm_hip_shard)");
    if (int st = ensure_buffers(h, true, false, true)) return st;
    if (d_b_rowmajor) *d_b_rowmajor = h->d_b;
    if (d_c) *d_c = h->d_c;
    return SPMM_HIP_OK;
}

int spmm_hip_destroy(spmm_hip_t *h) {
    if (!h) return SPMM_HIP_OK;
    multi_destroy(h);
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_plan(h);
    if (h->d_col) (void)hipFree(h->d_col);
    if (h->d_val) (void)hipFree(h->d_val);
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->side) {
        (void)hipStreamSynchronize(h->side);
        (void)hipStreamDestroy(h->side);
    }
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SPMM_HIP_OK;
}

int spmm_hip_debug_inspect(const int32_t *row_ptr, const int32_t *col_idx, int64_t m, int64_t ncols, int32_t T,
                           int32_t cap, int64_t win_cols, spmm_hip_inspection_t *out) {
    if (!row_ptr || !out || m < 0 || ncols < 0 || T < 1 || T > CAP || cap < T || cap > CAP || win_cols < 0)
        return fail(SPMM_HIP_ERR_ARG, "debug_inspect: bad arguments");
    std::memset(out, 0, sizeof(*out));
    Inspection in;
    if (win_cols > 0) {
        if (!col_idx && row_ptr[m] > 0) return fail(SPMM_HIP_ERR_ARG, "debug_inspect: col_idx NULL");
        if (!rows_sorted(row_ptr, col_idx, m)) return fail(SPMM_HIP_ERR_CSR, "debug_inspect: unsorted row");
        inspect_windows(row_ptr, col_idx, m, ncols, T, cap, win_cols, in);
    } else {
        inspect(row_ptr, m, T, cap, in);
        in.win_blk = {0, (int)in.blk.size()};
    }
    auto dup = [](const auto &v) {
        using E = typename std::decay_t<decltype(v)>::value_type;
        E *p = (E *)malloc(std::max<size_t>(v.size(), 1) * sizeof(E));
        if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(E));
        return p;
    };
    out->nv = (int64_t)in.vrow_ptr.size() - 1;
    out->nblk = (int64_t)in.blk.size();
    out->nwin = (int64_t)in.win_blk.size() - 1;
    out->nz = (int64_t)in.perm.size();
    out->nlong = (int64_t)in.long_rows.size();
    out->nslots = in.nslots;
    out->vrow_ptr = dup(in.vrow_ptr);
    out->vdest = dup(in.vdest);
    out->blk = (int32_t *)dup(in.blk);
    out->win_blk = dup(in.win_blk);
    out->long_rows = (int32_t *)dup(in.long_rows);
    out->perm = in.perm.empty() ? nullptr : dup(in.perm);
    return SPMM_HIP_OK;
}

int spmm_hip_debug_plan(const int32_t *row_ptr, const int32_t *col_idx, int64_t m, int64_t ncols, int32_t k,
                        int32_t dtype, int32_t mfma, int32_t gate_only, double *out) {
    if (!row_ptr || !out || m < 0 || ncols < 0 || k < 1 || (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32))
        return fail(SPMM_HIP_ERR_ARG, "debug_plan: bad arguments");
    if (m >= INT32_MAX || ncols >= INT32_MAX) return fail(SPMM_HIP_ERR_OVERFLOW, "debug_plan: m, ncols must fit int32");
    if (row_ptr[0] != 0) return fail(SPMM_HIP_ERR_CSR, "debug_plan: row_ptr[0] != 0");
    for (int64_t i = 0; i < m; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return fail(SPMM_HIP_ERR_CSR, "debug_plan: row_ptr not monotone");
    const int64_t nnz = row_ptr[m];
    if (nnz > 0 && !col_idx) return fail(SPMM_HIP_ERR_ARG, "debug_plan: col_idx NULL");
    // gate-only mode reads the columns of the gate's sampled rows only (the caller may fill no others): those are
    // range-checked, as every column is otherwise -- the gate indexes host arrays of ncols entries with them
    auto col_bad = [&](int64_t j) { return col_idx[j] < 0 || col_idx[j] >= ncols; };
    if (!gate_only) {
        for (int64_t j = 0; j < nnz; ++j)
            if (col_bad(j)) return fail(SPMM_HIP_ERR_CSR, "debug_plan: col_idx out of range");
    } else {
        bool bad = false;
        mfma_gate_tiles(m, [&](int64_t, int64_t r0, int64_t r1) {
            for (int64_t j = row_ptr[r0]; j < row_ptr[r1] && !bad; ++j) bad = col_bad(j);
        });
        if (bad) return fail(SPMM_HIP_ERR_CSR, "debug_plan: col_idx out of range (gate sample)");
    }
    spmm_hip_t h;                 // host-only view: no device state is touched
    h.dtype = dtype;
    h.vsize = dtype == SPMM_HIP_F64 ? 8 : 4;
    h.m = m, h.ncols = ncols, h.nnz = nnz;
    h.h_row_ptr.assign(row_ptr, row_ptr + m + 1);
    h.var.mfma = mfma;
    Draft d;
    if (int st = draft_plan(&h, k, col_idx, gate_only != 0, d)) return st;
    const Plan &p = d.pl;
    for (int i = 0; i < SPMM_HIP_PLAN_SLOTS; ++i) out[i] = 0.0;
    out[0] = d.gate_only ? (p.tile_mfma ? 2 : 0) : (p.ntile == 0 ? 0 : p.tile_mfma ? 2 : 1);
    out[1] = d.gate.verdict;
    out[2] = d.gate.r16;
    out[3] = d.gate.take;
    out[4] = d.gate.tile_nnz;
    out[5] = d.gate.chunks;
    out[6] = d.gate.max_chunks;
    out[7] = d.gate.t_on;
    out[8] = d.gate.t_off;
    out[9] = d.gate.sampled;
    out[10] = p.seq_max;
    out[11] = p.piece;
    out[12] = p.kw;
    out[13] = p.npanels;
    if (!d.gate_only) {
        out[14] = p.ntile;
        out[15] = (double)p.tile_nnz;
        out[16] = (double)p.tile_chunks;
        out[17] = (double)d.in.blk.size();
        out[18] = (double)d.in.long_rows.size();
        out[19] = (double)p.exact_rows;
        out[20] = p.lmax;
        out[21] = p.xcd;
        out[22] = p.nwin;
        const uint64_t fp = plan_fingerprint(d);
        out[24] = (double)(fp & 0xFFFFFFFFull);
        out[25] = (double)(fp >> 32);
    }
    out[23] = d.gate_only ? 1 : 0;
    out[26] = d.gate.tiles;
    out[27] = p.pair;
    out[28] = p.pair_reuse;
    out[29] = p.cap;
    return SPMM_HIP_OK;
}

int spmm_hip_debug_gate(int64_t m, int64_t nnz, int32_t k, int32_t kw, int32_t dtype, const double *sample,
                        double *out) {
    if (!sample || !out || m < 0 || nnz < 0 || k < 1 || kw < 1 || (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32))
        return fail(SPMM_HIP_ERR_ARG, "debug_gate: bad arguments");
    MfmaGate g;
    g.sampled = (int)sample[0];
    g.r16 = sample[1];
    g.take = sample[2];
    g.tiles = sample[3];
    g.tile_nnz = sample[4];
    g.chunks = sample[5];
    g.max_chunks = sample[6];
    // (the census's matrices are square: ncols = m)
    mfma_cost(g, m, m, nnz, k, kw, dtype == SPMM_HIP_F64 ? 8 : 4, gate_model(dtype == SPMM_HIP_F64 ? 8 : 4));
    out[0] = g.verdict;
    out[1] = g.t_on;
    out[2] = g.t_off;
    return SPMM_HIP_OK;
}

int spmm_hip_debug_tiles(const int32_t *row_ptr, const int32_t *col_idx, int64_t m, int64_t ncols, int32_t T,
                         int32_t rmax, int32_t uc, int32_t capa, double min_reuse, int32_t colmax, int32_t dmax,
                         spmm_hip_tiles_t *out) {
    if (!row_ptr || !out || m < 0 || ncols < 0 || T < 1 || rmax < 1 || uc < 1 || capa < 1 || capa > 65535 ||
        uc > 65536 || (!col_idx && m > 0 && row_ptr[m] > 0))
        return fail(SPMM_HIP_ERR_ARG, "debug_tiles: bad arguments");
    std::memset(out, 0, sizeof(*out));
    if (!rows_sorted(row_ptr, col_idx, m)) return fail(SPMM_HIP_ERR_CSR, "debug_tiles: unsorted row");
    TilePlan tp;
    build_tiles(row_ptr, col_idx, m, ncols, T, rmax, uc, capa, min_reuse, tp, colmax > 0 ? colmax : INT32_MAX,
                dmax > 0 ? dmax : INT32_MAX);
    if (!tile_tables_fit(tp))        // the plan would turn tiles off here (32-bit tile positions)
        return fail(SPMM_HIP_ERR_OVERFLOW, "debug_tiles: tile tables exceed the 32-bit position range");
    auto dup = [](const auto &v) {
        using E = typename std::decay_t<decltype(v)>::value_type;
        E *p = (E *)malloc(std::max<size_t>(v.size(), 1) * sizeof(E));
        if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(E));
        return p;
    };
    out->ntile = (int64_t)tp.tiles.size();
    out->nchunk = (int64_t)tp.chunks.size() - 1;
    out->ncol = (int64_t)tp.tcol.size();
    out->nseg = (int64_t)tp.tseg.size();
    out->nz = (int64_t)tp.perm.size();
    out->m = m;
    out->tiles = (int32_t *)dup(tp.tiles);
    out->chunks = (int32_t *)dup(tp.chunks);
    out->tcol = dup(tp.tcol);
    out->tseg = dup(tp.tseg);
    out->tlidx = dup(tp.tlidx);
    out->perm = dup(tp.perm);
    out->in_tile = dup(tp.in_tile);
    return SPMM_HIP_OK;
}

void spmm_hip_debug_tiles_free(spmm_hip_tiles_t *t) {
    if (!t) return;
    free(t->tiles);
    free(t->chunks);
    free(t->tcol);
    free(t->tseg);
    free(t->tlidx);
    free(t->perm);
    free(t->in_tile);
    std::memset(t, 0, sizeof(*t));
}

void spmm_hip_debug_free(spmm_hip_inspection_t *ins) {
    if (!ins) return;
    free(ins->vrow_ptr);
    free(ins->vdest);
    free(ins->blk);
    free(ins->win_blk);
    free(ins->long_rows);
    free(ins->perm);
    std::memset(ins, 0, sizeof(*ins));
}

#ifdef SPMM_TUNING
// Tuning build only (lib/libspmm_hip_tune.so, tools/tune_kernel.py): kernel variant + inspector overrides; the
// next run re-plans.  0 = policy default for seq_max / cap / panel_k / win_bytes (win_bytes < 0: no windows).
int spmm_hip_tune_select(spmm_hip_t *h, int u, int ntc, int dma, int buf, int seq_max, int cap, int panel_k,
                         int64_t win_bytes, int xcd, int lanes) {
    if (!h) return fail(SPMM_HIP_ERR_ARG, "tune_select: bad handle");
    h->var.u = u;
    h->var.ntc = ntc;
    h->var.dma = dma;
    h->var.buf = buf;
    h->var.seq_max = seq_max;
    h->var.cap = cap;
    h->var.panel_k = panel_k;
    h->var.win_bytes = win_bytes;
    h->var.xcd = xcd;
    h->var.lanes = lanes;
    h->var.tiles = env_int("SPMM_HIP_TUNE_TILES", 0);
    const int k = h->plan.k;
    h->plan.k = -1;
    return k > 0 ? spmm_hip_plan(h, k) : SPMM_HIP_OK;
}
#endif

}  // extern "C"
