// spmm_mfma.hpp -- gfx950 matrix-core (MFMA) tile kernel of the CSR SpMM engine.
//
// The sparse tile kernel (spmm_kernels.hpp, spmm_tile_kernel) reads one staged B row from LDS per nonzero and does
// VEC FMAs with it: the dense-row classes of the medium dataset sit at ~4 useful FMAs/clk/CU, bound by the LDS /
// L2 operand path.  Here every chunk of a tile is multiplied as a DENSE panel on the matrix
// cores,   C_tile[16 x 32 NP] += A_panel[16 x U] . B_chunk[U x 32 NP]   with v_mfma_f64_16x16x4_f64:
//   * a tile is 16 consecutive rows and belongs to ONE wave (four independent tiles per workgroup, no barrier);
//   * A_panel: the chunk's nonzeros scattered into the wave's zeroed LDS panel (row x chunk-local union column);
//     LDS operations of one wave execute in order, so the wave clears and refills its own panel without a barrier;
//   * B operand: one 16-byte load per lane per 4 union columns per 32-column sub-panel, straight from L2 into VGPRs:
//     lane l takes B columns 2j and 2j+1 (j = l & 15) of union column 4s + (l >> 4), feeding two MFMAs --
//     accumulator 0 owns the even B / C columns, accumulator 1 the odd ones -- so C is stored as 16-byte pairs;
//   * NP sub-panels of 32 columns per wave (NP = 2 for K >= 64): the A panel (entry loads, scatter,
//     LDS reads) is paid once per NP sub-panels;
//   * one MFMA does 1,024 FMAs from one f64 of A and one of B per lane (~16x less operand traffic per FMA than the
//     sparse kernel); the zero padding of the panel costs MFMA issue instead (useful fraction = panel density).
//
// Exactness.  The f64 MFMA accumulates its four products into C in k order, each one fused multiply-add (measured
// bit for bit against the reference chain, tests/test_gpu_mfma.py), so a tile row is the reference's left-to-right
// chain over its own columns with extra fma(0, b, acc) steps for the panel's empty cells.  Those extra steps are
// exact no-ops -- and the result does not depend on how the matrix cores treat subnormals -- whenever every nonzero
// operand the tile's MFMAs see (panel values a, B operand values b) has 2^-458 <= |x| <= 2^500:
//   * the chain starts at +0; a product is then 0 (an empty cell or a zero value: acc + (+-0) == acc, and +0 stays
//     +0) or at least 2^-916 in magnitude with its last bit >= 2^-1020; a step a*b + acc either cancels exactly
//     (+0, as in the reference) or lands at >= 2^-1021 in magnitude (|acc| near |a*b| has its last bit >= 2^-969,
//     otherwise one term dominates) -- so no step underflows, none produces -0 or a subnormal, none overflows
//     (<= 2048 products of <= 2^1000), and an empty cell never meets a -0 accumulator (fma(+0, b, -0) would give
//     +0 where the reference keeps -0).
// The check is made on the operands as they enter the MFMAs (no extra registers live); a wave that meets an operand
// outside the range -- Inf/NaN in B, subnormal or extreme values: adversarial data only -- recomputes its whole tile
// by the sparse chain over the real entries with IEEE FMAs (exactly the reference's operations), from +0.  Rows with
// a repeated column (duplicate .mtx entries) never reach this kernel (the inspector keeps them out).
//
// Per-wave pipeline, chunk c: A(c) from the panel into VGPRs; clear chunk c's cells, scatter chunk c+1's entries
// (loaded during chunk c-1); issue the entry loads of chunk c+2; the MFMAs of chunk c (operands range-checked), each
// k step's B registers reloaded with chunk c+1's operand as soon as its MFMAs have issued; the union-column loads of
// chunk c+2.  VGPRs: 154 (NP = 1, 3 waves per SIMD) / 218 (NP = 2, 2 waves per SIMD), no spills.
//
// Tables (inspector build_tiles with 16-row tiles; spmm_engine.hip):
//   tiles[t]   = {first C row, rows (<= 16), first chunk, chunks}
//   tchunk[c]  = {-, columns U, first entry, -}; sentinel after the last chunk
//   tcolT[c*48 + g*12 + s] = B row of chunk c's union column 4s + g (padded with a valid row past U)
//   tval[e]    = chunk entries, row by row (padding +0);  tpos[e] = panel cell row * 49 + column (padding: trash)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spmm {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int MFMA_UC = 48;                    // union columns per chunk
constexpr int MFMA_KS = MFMA_UC / 4;           // k steps per chunk
constexpr int MFMA_PST = MFMA_UC + 1;          // panel row stride (doubles; odd: rows spread over the LDS banks)
constexpr int MFMA_ROWS = 16;                  // rows per tile (one wave)
constexpr int MFMA_TRASH = MFMA_ROWS * MFMA_PST;
constexpr int MFMA_PSZ = MFMA_TRASH + 2;       // one wave's panel (+ trash cell)
constexpr int MFMA_CAPA = 512;                 // entries per chunk (8 per lane)
constexpr int MFMA_NPE = MFMA_CAPA / 64;

// operand outside the exact-chain range (see the header): nonzero and |x| < 2^-458, |x| > 2^500, Inf or NaN
__device__ __forceinline__ bool mfma_operand_bad(double x) {
    const double ax = __builtin_fabs(x);
    return !(ax >= 0x1p-458 && ax <= 0x1p500) && x != 0.0;
}
template <bool XCD, int NP>
__global__ __launch_bounds__(256, NP == 1 ? 3 : 2) void spmm_mfma_tile_kernel(const int4 *__restrict__ tiles,
                                                                              int ntiles,
                                                                              const int4 *__restrict__ tchunk,
                                                                              const int32_t *__restrict__ tcolT,
                                                                              const double *__restrict__ tval,
                                                                              const uint16_t *__restrict__ tpos,
                                                                              const double *__restrict__ B,
                                                                              uint32_t b_bytes, double *__restrict__ C,
                                                                              int ld) {
    __shared__ __attribute__((aligned(16))) double spanel[4 * MFMA_PSZ];
    const int wave = threadIdx.x / 64, l = threadIdx.x % 64;
    const int wg = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int t = __builtin_amdgcn_readfirstlane(wg * 4 + wave);
    if (t >= ntiles) return;
    const int4 tl = tiles[t];
    double *P = spanel + wave * MFMA_PSZ;
    for (int i = l; i < MFMA_PSZ; i += 64) P[i] = 0.0;

    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t ldb = (uint32_t)ld * 8u, lane_off = (uint32_t)(l & 15) * 16u;
    const int g = l >> 4;

    f64x4 acc[NP][2];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p][0] = acc[p][1] = f64x4{0.0, 0.0, 0.0, 0.0};
    i32x4 bo[NP][MFMA_KS];
    int tcn[MFMA_KS];
    double ev[MFMA_NPE];
    int ep[MFMA_NPE], hc[MFMA_NPE];
    int ne = 0;
    auto load_tcol = [&](int c) {                 // this lane's 12 union columns of chunk c (3 x 16 B)
        const i32x4 *p = reinterpret_cast<const i32x4 *>(tcolT + (size_t)(tl.z + c) * MFMA_UC + g * MFMA_KS);
#pragma unroll
        for (int q = 0; q < MFMA_KS / 4; ++q) {
            const i32x4 v = p[q];
            tcn[4 * q] = v.x, tcn[4 * q + 1] = v.y, tcn[4 * q + 2] = v.z, tcn[4 * q + 3] = v.w;
        }
    };
    auto load_b1 = [&](int st) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
            bo[p][st] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)tcn[st] * ldb + lane_off + 256u * p, 0, 0);
    };
    auto load_e = [&](int c) {
        const int4 ch = tchunk[tl.z + c], cn = tchunk[tl.z + c + 1];
        ne = cn.z - ch.z;
#pragma unroll
        for (int j = 0; j < MFMA_NPE; ++j) {
            const int e = min(j * 64 + l, ne - 1);
            ev[j] = __builtin_nontemporal_load(tval + ch.z + e);
            ep[j] = (int)__builtin_nontemporal_load(tpos + ch.z + e);
        }
    };
    auto scatter = [&]() {
#pragma unroll
        for (int j = 0; j < MFMA_NPE; ++j) {
            const int cell = j * 64 + l < ne ? ep[j] : MFMA_TRASH;
            P[cell] = ev[j];
            hc[j] = cell;
        }
    };
    // chunk c by the sparse chain (IEEE FMAs over the chunk's real entries in order, from the accumulators): an
    // entry of row r updates this lane's outputs when r % 4 == g (the fallback of a tile with an operand outside the
    // exact range)
    auto sparse_chunk = [&](int c) {
        const int4 ch = tchunk[tl.z + c], cn = tchunk[tl.z + c + 1];
        double x[NP][8];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int i = 0; i < 4; ++i) x[p][i] = acc[p][0][i], x[p][4 + i] = acc[p][1][i];
#pragma unroll 1
        for (int e = ch.z; e < cn.z; ++e) {
            const int cell = (int)tpos[e];
            const int r = cell / MFMA_PST, k = cell % MFMA_PST;
            if (cell == MFMA_TRASH || (r & 3) != g) continue;
            const int row = tcolT[(size_t)(tl.z + c) * MFMA_UC + (k & 3) * MFMA_KS + (k >> 2)];
            const double av = tval[e];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)row * ldb + lane_off + 256u * p, 0, 0);
                double bb[2];
                __builtin_memcpy(bb, &v, 16);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q == (r >> 2)) {
                        x[p][q] = __builtin_fma(av, bb[0], x[p][q]);
                        x[p][4 + q] = __builtin_fma(av, bb[1], x[p][4 + q]);
                    }
            }
        }
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[p][0][i] = x[p][i], acc[p][1][i] = x[p][4 + i];
    };

    // prologue: chunk 0 in the panel, B operand of chunk 0, entries and union columns of chunk 1
    load_tcol(0);
#pragma unroll
    for (int st = 0; st < MFMA_KS; ++st) load_b1(st);
    load_e(0);
    scatter();
    load_e(min(1, tl.w - 1));
    load_tcol(min(1, tl.w - 1));
    bool bad = false;
    for (int c = 0; c < tl.w; ++c) {
        const int ns = (tchunk[tl.z + c].y + 3) >> 2;
        double a[MFMA_KS];
        const double *pa = P + (l & 15) * MFMA_PST + g;
#pragma unroll
        for (int st = 0; st < MFMA_KS; ++st) a[st] = pa[4 * st];
#pragma unroll
        for (int j = 0; j < MFMA_NPE; ++j) P[hc[j]] = 0.0;
        if (c + 1 < tl.w) scatter();
        load_e(min(c + 2, tl.w - 1));
#pragma unroll
        for (int st = 0; st < MFMA_KS; ++st) {
            if (st < ns) {
                bad |= mfma_operand_bad(a[st]);
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    double bb[2];
                    __builtin_memcpy(bb, &bo[p][st], 16);
                    bad |= mfma_operand_bad(bb[0]) || mfma_operand_bad(bb[1]);
                    acc[p][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[st], bb[0], acc[p][0], 0, 0, 0);
                    acc[p][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[st], bb[1], acc[p][1], 0, 0, 0);
                }
            }
            load_b1(st);                           // chunk c+1's operand (tcn holds its columns)
        }
        if (__builtin_amdgcn_ballot_w64(bad)) break;
        load_tcol(min(c + 2, tl.w - 1));
    }
    if (__builtin_amdgcn_ballot_w64(bad)) {      // an operand outside the exact range: the tile by the sparse chain
#pragma unroll
        for (int p = 0; p < NP; ++p) acc[p][0] = acc[p][1] = f64x4{0.0, 0.0, 0.0, 0.0};
        for (int c = 0; c < tl.w; ++c) sparse_chunk(c);
    }
    const int c0 = 2 * (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = g + 4 * i;
        if (r < tl.y) {
            double *p = C + (size_t)(tl.x + r) * ld + c0;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                __builtin_nontemporal_store(acc[q][0][i], p + 32 * q);
                __builtin_nontemporal_store(acc[q][1][i], p + 32 * q + 1);
            }
        }
    }
}

}  // namespace spmm
