// spmm_mfma.hpp -- gfx950 matrix-core (MFMA) tile kernel of the CSR SpMM engine.
//
// The sparse tile kernel (spmm_kernels.hpp, spmm_tile_kernel) reads one staged B row from LDS per nonzero and does
// VEC FMAs with it: the dense-row classes of the medium dataset sit at ~4 useful FMAs/clk/CU, bound by the LDS /
// L2 operand path.  Here every chunk of a tile is multiplied as a DENSE panel on the matrix
// cores,   C_tile[16 x 32 NP] += A_panel[16 x U] . B_chunk[U x 32 NP]   with v_mfma_f64_16x16x4_f64 (fp64) or
// v_mfma_f32_16x16x4_f32 (fp32):
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
// Exactness.  Both MFMAs accumulate their four products into C in k order, each one fused multiply-add (measured
// bit for bit, tools/mfma_chain_probe.py: 25,600 of 25,600 outputs each; and against the reference chain,
// tests/test_gpu_mfma.py), so a tile row is the reference's left-to-right
// chain over its own columns with extra fma(0, b, acc) steps for the panel's empty cells.  Those extra steps are
// exact no-ops -- and the result does not depend on how the matrix cores treat subnormals -- whenever every nonzero
// operand has 2^-458 <= |x| < 2^500 (fp32: 2^-40 <= |x| < 2^58, the same argument with 24-bit significands and a
// 2^-126 normal floor; fp64 figures below):
//   * the chain starts at +0; a product is then 0 (an empty cell or a zero value: acc + (+-0) == acc, and +0 stays
//     +0) or at least 2^-916 in magnitude with its last bit >= 2^-1020; a step a*b + acc either cancels exactly
//     (+0, as in the reference) or lands at >= 2^-1021 in magnitude (|acc| near |a*b| has its last bit >= 2^-969,
//     otherwise one term dominates) -- so no step underflows or produces a subnormal, no -0 ever appears, and an
//     empty cell never meets a -0 accumulator (fma(+0, b, -0) would give +0 where the reference keeps -0);
//   * no product reaches 2^1000 and no row of <= 2048 of them overflows, and Inf / NaN (a panel zero times them
//     makes a NaN the reference does not have) are outside the range.
// The range is checked outside the MFMA loop: A's values when the plan is built and whenever they are updated
// (mflag[0]), B by mfma_range_kernel on the side stream beside the tile kernel (mflag[1] == the launch's sequence
// number).  When either is set -- adversarial data only -- mfma_fixup_kernel, after both, recomputes every tile by
// the sparse chain over the real entries with IEEE FMAs from +0, exactly the reference's operations.  Rows with a
// repeated column (duplicate .mtx entries) never reach this kernel.
//
// Per-wave pipeline, chunk c: A(c) from the panel into VGPRs; clear chunk c's cells, scatter chunk c+1's entries
// (loaded during chunk c-1); issue the entry loads of chunk c+2; the MFMAs of chunk c, each
// k step's B registers reloaded with chunk c+1's operand as soon as its MFMAs have issued; the union-column loads of
// chunk c+2.
//
// Tables (inspector build_tiles with 16-row tiles; spmm_engine.hip):
//   tiles[t]   = {first C row, rows (<= 16), first chunk, chunks}
//   tchunk[c]  = {-, columns U, first entry, -}; sentinel after the last chunk
//   tcolT[c*48 + g*12 + s] = B row of chunk c's union column 4s + g (padded with a valid row past U)
//   tpos[e]    = panel cell (row * 49 + column; padding: trash) of the chunk's entry e, row by row; a chunk holds a
//                multiple of 8 entries (ne = 8 nl) and lane l < nl takes entries 8l .. 8l+7 with ONE 16-byte load
//   tval[...]  = their values (padding +0), permuted within the chunk so that lane l's 8 values are 16-byte pieces
//                of 16/sizeof(T)-entry runs: entry 8l + j sits at mfma_val_pos<T>(8l + j, nl) (2 / 4 loads per lane,
//                fp64 / fp32, each wave instruction contiguous) -- 5 (fp64) or 3 (fp32) vector-memory instructions per
//                chunk for the entries instead of 16 (the TA issue rate, not bytes, bounds them: r05e PMC)
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

// Position of chunk entry s (lane s / 8, its j = s % 8) in the chunk's value block of 8 nl entries (see tval above)
template <typename T>
__host__ __device__ inline int mfma_val_pos(int s, int nl) {
    constexpr int VPL = 16 / (int)sizeof(T);
    const int l = s >> 3, j = s & 7;
    return VPL * nl * (j / VPL) + VPL * l + (j % VPL);
}

// Per value type: the 16x16x4 MFMA, its accumulator, the B operand piece a lane loads (columns 2j, 2j+1 of a
// 32-column sub-panel: 16 B fp64 / 8 B fp32), the C/D row map (f64: row = g + 4i; f32: row = 4g + i, g = lane >> 4 --
// measured, tools/mfma_chain_probe.py) and the exactness range (see the header): a nonzero operand needs a frexp
// exponent >= MIN_EXP, |x| >= 2^-458 fp64 / 2^-40 fp32 (zero has exponent 0, a subnormal far less).  The kernel
// keeps the smallest exponent a lane has fed to its MFMAs (one v_frexp_exp + one v_min per operand).
template <typename T> struct MfmaT;
template <> struct MfmaT<double> {
    typedef f64x4 acc_t;
    typedef i32x4 bop_t;
    static constexpr int MIN_EXP = -457, MAX_EXP = 500;
    __device__ static int fexp(double x) { return __builtin_amdgcn_frexp_exp(x); }
    __device__ static acc_t mfma(double a, double b, acc_t c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
    __device__ static bop_t load(__amdgpu_buffer_rsrc_t rs, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0); }
    __device__ static int row(int g, int i) { return g + 4 * i; }
    __device__ static bool owns(int r, int g) { return (r & 3) == g; }
    __device__ static int slot(int r) { return r >> 2; }
    __device__ static double fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
};
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
template <> struct MfmaT<float> {
    typedef f32x4 acc_t;
    typedef i32x2 bop_t;
    static constexpr int MIN_EXP = -39, MAX_EXP = 58;
    __device__ static int fexp(float x) { return __builtin_amdgcn_frexp_expf(x); }
    __device__ static acc_t mfma(float a, float b, acc_t c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
    __device__ static bop_t load(__amdgpu_buffer_rsrc_t rs, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0); }
    __device__ static int row(int g, int i) { return 4 * g + i; }
    __device__ static bool owns(int r, int g) { return (r >> 2) == g; }
    __device__ static int slot(int r) { return r & 3; }
    __device__ static float fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
};

// Waves per SIMD the register budget allows: a whole chunk of B operands in flight (R = 12) costs 4 VGPRs per slot and
// sub-panel; a ring of R < 12 slots (the operand of step s + R loaded once step s's MFMAs have issued) frees them.
template <typename T, int NP, int R>
constexpr int mfma_waves() {
    return sizeof(T) == 4 ? (R < MFMA_KS ? 4 : 3) : (NP == 1 ? (R < MFMA_KS ? 4 : 3) : (R < MFMA_KS ? 3 : 2));
}

// No range check here: mfma_fixup_kernel recomputes every tile when an operand lies outside the exact range
template <typename T, bool XCD, int NP, int R = MFMA_KS>
__global__ __launch_bounds__(256, (mfma_waves<T, NP, R>())) void spmm_mfma_tile_kernel(
    const int4 *__restrict__ tiles, int ntiles, const int4 *__restrict__ tchunk, const int32_t *__restrict__ tcolT,
    const T *__restrict__ tval, const uint16_t *__restrict__ tpos, const T *__restrict__ B, uint32_t b_bytes,
    T *__restrict__ C, int ld) {
    static_assert(R >= 1 && R <= MFMA_KS && MFMA_KS % R == 0, "ring slots");
    using M = MfmaT<T>;
    typedef typename M::acc_t acc_t;
    typedef typename M::bop_t bop_t;
    constexpr uint32_t SUB = 32u * sizeof(T);   // bytes of one 32-column sub-panel of a B row
    __shared__ __attribute__((aligned(16))) T spanel[4 * MFMA_PSZ];
    const int wave = threadIdx.x / 64, l = threadIdx.x % 64;
    const int wg = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int t = __builtin_amdgcn_readfirstlane(wg * 4 + wave);
    if (t >= ntiles) return;
    const int4 tl = tiles[t];
    T *P = spanel + wave * MFMA_PSZ;
    for (int i = l; i < MFMA_PSZ; i += 64) P[i] = T(0);

    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t ldb = (uint32_t)ld * (uint32_t)sizeof(T), lane_off = (uint32_t)(l & 15) * 2u * (uint32_t)sizeof(T);
    const int g = l >> 4;

    acc_t acc[NP][2];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p][0] = acc[p][1] = acc_t{T(0), T(0), T(0), T(0)};
    bop_t bo[NP][R];
    int tcn[MFMA_KS];       // R = 12: union columns of the chunk whose B operand is being loaded (c+1 in iteration c)
    int tn = 0;             // lane < 48: one union column of chunk c+2, fetched an iteration ahead
    constexpr int VPL = 16 / (int)sizeof(T);     // values per 16-byte piece
    typedef T tv __attribute__((ext_vector_type(VPL)));
    tv ev[8 / VPL];                              // this lane's 8 entries: values ...
    i32x4 ep;                                    // ... and panel cells (8 x u16)
    int hc[8];
    int ne = 0;
    // Vector-memory results are waited for in issue order (s_waitcnt vmcnt): a wait for one load drags every older load
    // with it, and the compiler's waits are static, sized for every path into a block.  So a register the loop's B
    // loads address with must never be a vector-memory destination on any path: the union columns go global -> VGPR
    // (tn, fetched at the TOP of iteration c for chunk c+2, ahead of the B loads issued during its MFMAs) -> LDS (end
    // of the iteration: waits only for loads a whole iteration old) -> the B loads' addresses (LDS reads).  The
    // prologue issues its loads in the loop's order, so the first iteration's waits are the steady state's.
    // (Round 4's kernel fetched the columns after the B loads: the next chunk's first B load waited for all of them,
    // one exposed memory latency per chunk.)
    __shared__ __attribute__((aligned(16))) int stc[4 * 2 * MFMA_UC];   // per wave: columns of two chunks
    int *TC = stc + wave * 2 * MFMA_UC;
    auto fetch_tcol = [&](int c) {
        if (l < MFMA_UC) tn = __builtin_nontemporal_load(tcolT + (size_t)(tl.z + c) * MFMA_UC + l);
    };
    auto put_tcol = [&](int c) {
        if (l < MFMA_UC) TC[(c & 1) * MFMA_UC + l] = tn;
    };
    auto take_tcol = [&](int c) {                 // this lane's 12 columns of chunk c (its k-step group g)
        const i32x4 *p = reinterpret_cast<const i32x4 *>(TC + (c & 1) * MFMA_UC + g * MFMA_KS);
#pragma unroll
        for (int q = 0; q < MFMA_KS / 4; ++q) {
            const i32x4 v = p[q];
            tcn[4 * q] = v.x, tcn[4 * q + 1] = v.y, tcn[4 * q + 2] = v.z, tcn[4 * q + 3] = v.w;
        }
    };
    // B operand of (chunk c, step st) into ring slot st % R; R = 12 addresses with tcn (chunk c's columns, taken at
    // the top of the iteration), a ring reads each column from LDS when it loads
    auto load_b = [&](int c, int st) {
        const int col = R == MFMA_KS ? tcn[st] : TC[(c & 1) * MFMA_UC + g * MFMA_KS + st];
#pragma unroll
        for (int p = 0; p < NP; ++p) bo[p][st % R] = M::load(rs, (uint32_t)col * ldb + lane_off + SUB * p);
    };
    auto load_e = [&](int c) {                    // 16-byte loads only (lanes past the entries reload the last 8)
        const int4 ch = tchunk[tl.z + c], cn = tchunk[tl.z + c + 1];
        ne = cn.z - ch.z;
        const int nl = ne >> 3, lq = min(l, nl - 1);
        ep = __builtin_nontemporal_load(reinterpret_cast<const i32x4 *>(tpos + ch.z) + lq);
#pragma unroll
        for (int q = 0; q < 8 / VPL; ++q)
            ev[q] = __builtin_nontemporal_load(reinterpret_cast<const tv *>(tval + ch.z + VPL * nl * q) + lq);
    };
    auto scatter = [&]() {
        const bool on = 8 * l < ne;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int cell = on ? (int)((uint32_t)ep[j >> 1] >> (16 * (j & 1)) & 0xFFFFu) : MFMA_TRASH;
            P[cell] = ev[j / VPL][j % VPL];
            hc[j] = cell;
        }
    };
    // prologue: chunk 0 in the panel; then, in the loop's order, chunk 1's columns, chunk 1's entries, the first R
    // steps' B operand of chunk 0, chunk 1's columns into LDS
    fetch_tcol(0);
    put_tcol(0);
    load_e(0);
    scatter();
    fetch_tcol(min(1, tl.w - 1));
    load_e(min(1, tl.w - 1));
    if (R == MFMA_KS) take_tcol(0);
#pragma unroll
    for (int st = 0; st < R; ++st) load_b(0, st);
    put_tcol(1);
    for (int c = 0; c < tl.w; ++c) {
        const int ns = (tchunk[tl.z + c].y + 3) >> 2;
        fetch_tcol(min(c + 2, tl.w - 1));
        if (R == MFMA_KS) take_tcol(c + 1);        // chunk c+1's columns (its B operand loads during these MFMAs)
        T a[MFMA_KS];
        const T *pa = P + (l & 15) * MFMA_PST + g;
#pragma unroll
        for (int st = 0; st < MFMA_KS; ++st) a[st] = pa[4 * st];
#pragma unroll
        for (int j = 0; j < 8; ++j) P[hc[j]] = T(0);
        if (c + 1 < tl.w) scatter();             // chunk c+1's entries (ev / ep, loaded an iteration ago) ...
        load_e(min(c + 2, tl.w - 1));             // ... before the registers take chunk c+2's
#pragma unroll
        for (int st = 0; st < MFMA_KS; ++st) {
            if (st < ns) {
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    T bb[2];
                    __builtin_memcpy(bb, &bo[p][st % R], 2 * sizeof(T));
                    acc[p][0] = M::mfma(a[st], bb[0], acc[p][0]);
                    acc[p][1] = M::mfma(a[st], bb[1], acc[p][1]);
                }
            }
            // the slot just read takes step st + R: of this chunk, or of the next
            if (st + R < MFMA_KS) load_b(c, st + R);
            else load_b(c + 1, st + R - MFMA_KS);
        }
        put_tcol(c + 2);                           // buffer (c & 1): chunk c's columns are no longer read
    }
    const int c0 = 2 * (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = M::row(g, i);
        if (r < tl.y) {
            T *p = C + (size_t)(tl.x + r) * ld + c0;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                __builtin_nontemporal_store(acc[q][0][i], p + 32 * q);
                __builtin_nontemporal_store(acc[q][1][i], p + 32 * q + 1);
            }
        }
    }
}

// Exact-range check of B for the matrix-core tiles (mflag[1]; on the side stream beside the tile kernel): any value
// with a frexp exponent outside [MIN_EXP, MAX_EXP] other than +-0 -- subnormals, tiny or huge values, Inf, NaN
// (frexp gives NaN / Inf the exponent 0, so those are caught by the finiteness test) -- stores seq into *flag.
// 16-byte loads over n values.
template <typename T>
__global__ __launch_bounds__(256) void mfma_range_kernel(const T *__restrict__ B, int64_t n, int *__restrict__ flag,
                                                         int seq) {
    using M = MfmaT<T>;
    constexpr int V = 16 / (int)sizeof(T);
    typedef T tv __attribute__((ext_vector_type(V)));
    bool bad = false;
    const int64_t nv = n / V, stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
        const tv v = reinterpret_cast<const tv *>(B)[i];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int e = M::fexp(v[j]);
            bad |= (v[j] != T(0) && (e < M::MIN_EXP || e > M::MAX_EXP)) || !__builtin_isfinite(v[j]);
        }
    }
    for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const T x = B[i];
        const int e = M::fexp(x);
        bad |= (x != T(0) && (e < M::MIN_EXP || e > M::MAX_EXP)) || !__builtin_isfinite(x);
    }
    if (__builtin_amdgcn_ballot_w64(bad) && (threadIdx.x & 63) == 0) atomicExch(flag, seq);
}

// The tiles of a launch with an operand outside the exact range (mflag[0]: A's values, set at plan time or by a value
// update; mflag[1] == seq: this launch's B, mfma_range_kernel) recomputed after the tile kernel, over all K columns, by
// the sparse chain over each row's real entries with IEEE FMAs from +0 -- exactly the reference's operations.  Every
// other launch leaves at its first instruction.  One wave per tile (grid-stride); lane l owns C columns 2j, 2j+1 of
// each 32-column sub-panel (j = l & 15) for the rows r with M::owns(r, l >> 4), as the tile kernel's accumulators.
template <typename T>
__global__ __launch_bounds__(256) void mfma_fixup_kernel(
    const int4 *__restrict__ tiles, int ntiles, const int4 *__restrict__ tchunk, const int32_t *__restrict__ tcolT,
    const T *__restrict__ tval, const uint16_t *__restrict__ tpos, const T *__restrict__ B, T *__restrict__ C, int ld,
    int K, const int *__restrict__ mflag, int seq) {
    using M = MfmaT<T>;
    if (__builtin_amdgcn_readfirstlane(mflag[0] == 0 && mflag[1] != seq)) return;
    const int l = threadIdx.x % 64, g = l >> 4, c0 = 2 * (l & 15);
    const int nw = (int)gridDim.x * 4;
    for (int t = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)threadIdx.x / 64); t < ntiles; t += nw) {
        const int4 tl = tiles[t];
        for (int k0 = 0; k0 + 32 <= K; k0 += 32) {
            T x[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = T(0);
            for (int c = 0; c < tl.w; ++c) {
                const int4 ch = tchunk[tl.z + c], cn = tchunk[tl.z + c + 1];
                const int nl = (cn.z - ch.z) >> 3;
                for (int e = ch.z; e < cn.z; ++e) {
                    const int cell = (int)tpos[e];
                    const int r = cell / MFMA_PST, k = cell % MFMA_PST;
                    if (cell == MFMA_TRASH || !M::owns(r, g)) continue;
                    const int row = tcolT[(size_t)(tl.z + c) * MFMA_UC + (k & 3) * MFMA_KS + (k >> 2)];
                    const T av = tval[ch.z + mfma_val_pos<T>(e - ch.z, nl)];
                    const T *b = B + (size_t)row * ld + k0 + c0;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (q == M::slot(r)) {
                            x[q] = M::fma(av, b[0], x[q]);
                            x[4 + q] = M::fma(av, b[1], x[4 + q]);
                        }
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = M::row(g, i);
                if (r < tl.y) {
                    T *p = C + (size_t)(tl.x + r) * ld + k0 + c0;
                    p[0] = x[i];
                    p[1] = x[4 + i];
                }
            }
        }
    }
}

}  // namespace spmm
