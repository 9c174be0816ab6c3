// spmm_staged.hpp -- gfx950 kernel for STAGED ROWS: whole rows of tens to a few thousand nonzeros.
//
// Restates the reference's inner loop (benchmark_code/CPU/AMD/spmv_code_bench/spmm_kernel_csr.cpp:84-92) for rows
// the row-block kernel serves badly: there a row is one G-lane group with U gathers in flight, so a 500-nonzero row
// is ~32 dependent gather round trips and a 2,048-nonzero block of such rows keeps one wave of its four busy -- a
// small matrix (698 x 500: 175 blocks) leaves most of the chip's gather slots empty, and a large one drains every
// group's batch before its next.  Here a workgroup owns R whole rows and ALL 256 lanes gather:
//   * chunk c of the workgroup = nonzeros [c*CH, c*CH + CH) of each of its R rows (CH = NE / R, NE = 16 KiB of B
//     rows); lane t gathers the 16-byte pieces t, t+256, ... of the chunk's B rows (GPT per lane) into VGPRs,
//     two chunks ahead, and writes them to one of two LDS chunk buffers when the chunk before has been folded;
//   * consumer lanes: one lane per (row, VC columns); lane (row s, column n) folds the chunk's nonzeros of row s in
//     CSR order, acc = fma(a[j], B[col[j]][n], acc) from j = row start to row end -- the reference's chain, one per
//     C element, carried in a register across chunks, so every row is bit-identical to the reference.
// Loads whose entry lies past its row's end get a byte offset past the buffer's extent: the buffer unit returns
// zeros without touching memory, and every lane issues the same load sequence (static vmcnt waits).
// Order of one step (chunk c in LDS buffer c&1): columns of chunk c+D+2 -> VGPRs, gathers of chunk c+D -> VGPRs, fold
// chunk c, chunk c+1's gathers -> LDS buffer (c+1)&1, barrier.  While chunk c is folded, chunks c+1 .. c+D are in
// flight (D = 3); the columns are fetched two steps before their gathers so each wait covers only what the step
// needs.  (D = 2 with the columns one step ahead ran 1.5-3x slower than the row kernel: each step then waits ~2/3
// of a loaded L2 round trip for 16 KiB.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spmm_kernels.hpp"

namespace spmm {

constexpr int STG_BUFB = 16384;   // LDS bytes of one chunk's B rows (two chunk buffers per workgroup)
constexpr int STG_RMAX = 32;      // rows per workgroup at most
constexpr uint32_t STG_OOB = 0xFFFFFFF0u;   // buffer byte offset past every extent: the load returns zeros
constexpr int STG_D = 3;           // chunks whose gathers are in flight while one is folded
constexpr int STG_UN = 6;          // steps per loop round: lcm(STG_D, 3 column sets, 2 LDS buffers)
constexpr int STG_FU = 4;          // fold unroll (LDS reads issued ahead of their FMAs)

// Lane geometry of a panel whose B rows are SB bytes (SB in {64, 128, 256, 512, 1024})
template <typename T, int SB>
struct StagedShape {
    static constexpr int KW = SB / (int)sizeof(T);                 // panel columns
    static constexpr int CL = KW < 64 ? KW : 64;                   // consumer lanes per row
    static constexpr int VC = KW / CL;                             // columns per consumer lane
    static constexpr int RW = 64 / CL;                             // rows per wave
    static constexpr int LPE = SB / 16;                            // 16-byte pieces per B row
    static constexpr int NE = STG_BUFB / SB;                      // entries per chunk (all rows)
    static constexpr int GPT = STG_BUFB / (16 * WG);              // gathers per lane per chunk
    static constexpr int RM0 = 4 * RW < NE ? 4 * RW : NE;
    static constexpr int RMAX = RM0 < STG_RMAX ? RM0 : STG_RMAX; // rows per workgroup at most
    static_assert(SB % 16 == 0 && SB >= 64 && SB <= 1024 && (SB & (SB - 1)) == 0, "B row bytes");
    static_assert(GPT * 16 * WG == STG_BUFB && NE <= WG && WG % LPE == 0, "chunk geometry");
};

// wg[b] = {first nonzero, end nonzero} of workgroup b's rows; slot[b*R + s] = {C row (-1 = none), first nonzero,
// nonzeros, 0} of its row slot s (R = 2^rlog).  B, C: the panel's first column; ld their row stride (K); b_bytes B's
// extent from B on (below 4 GiB - 256, checked at plan).
template <typename T, int SB, bool NTC, bool XCD>
__global__ __launch_bounds__(WG, 4) void spmm_staged_rows_kernel(const int32_t *__restrict__ col_idx,
                                                                 const T *__restrict__ vals,
                                                                 const int2 *__restrict__ wg,
                                                                 const int4 *__restrict__ slot_tab, int rlog,
                                                                 const T *__restrict__ B, T *__restrict__ C, int ld,
                                                                 uint32_t b_bytes) {
    using S = StagedShape<T, SB>;
    using V = vec<T, S::VC>;
    __shared__ __attribute__((aligned(16))) char s_b[2][STG_BUFB];
    __shared__ __attribute__((aligned(16))) T s_v[2][WG];   // entry values (lanes >= NE: unread copies)
    __shared__ int s_beg[STG_RMAX], s_len[STG_RMAX];   // row slots: first nonzero (workgroup-relative), length

    const int tid = threadIdx.x;
    const int b = XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int R = 1 << rlog;
    const int clog = __builtin_ctz((unsigned)S::NE) - rlog;      // CH = NE / R
    const int CH = 1 << clog;
    const int2 rng = wg[b];                                      // uniform: scalar loads
    if (tid < R) {
        const int4 sl = slot_tab[b * R + tid];
        s_beg[tid] = sl.y - rng.x;                               // relative to the workgroup's first nonzero
        s_len[tid] = sl.z;
    }
    __syncthreads();
    int lmax = 0;
    for (int s = 0; s < R; ++s) lmax = max(lmax, s_len[s]);
    const int nch = (lmax + CH - 1) >> clog;

    // the workgroup's columns and values as buffer resources (offsets relative to its first nonzero)
    const uint32_t nz = (uint32_t)(rng.y - rng.x);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)(col_idx + rng.x), (short)0,
                                                                        (int)(nz * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void *)(vals + rng.x), (short)0,
                                                                        (int)(nz * (uint32_t)sizeof(T)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)b_bytes, 0x00020000);
    const uint32_t rowb = (uint32_t)ld * (uint32_t)sizeof(T);

    // producer pieces: piece p = tid + 256 u is byte 16 p of the chunk image = entry p / LPE (row slot e >> clog,
    // position e & (CH-1) in the chunk), 16-byte column piece p % LPE
    int pbeg[S::GPT], plen[S::GPT];
    const uint32_t qoff = (uint32_t)(tid % S::LPE) * 16u;       // WG is a multiple of LPE: the same for every u
#pragma unroll
    for (int u = 0; u < S::GPT; ++u) {
        const int e = (tid + WG * u) / S::LPE, s = e >> clog, j = e & (CH - 1);
        pbeg[u] = s_beg[s] + j;
        plen[u] = s_len[s] - j;                                  // entries of the row from this position on
    }
    // values: lane t < NE loads entry t's value (every lane issues the load; lanes >= NE repeat entry t % NE)
    const int ve = tid % S::NE, vs = ve >> clog, vj = ve & (CH - 1);
    const int vbeg = s_beg[vs] + vj, vlen = s_len[vs] - vj;

    // in flight: the gathers of STG_D chunks (VGPR sets by chunk % STG_D) and the columns of the two chunks after
    // them (sets by chunk % 3)
    int kc[3][S::GPT];
    i32x4 g[STG_D][S::GPT];
    T va[STG_D];
    auto load_cols = [&](int c, int (&k)[S::GPT]) {
#pragma unroll
        for (int u = 0; u < S::GPT; ++u) {
            const uint32_t off = c * CH < plen[u] ? (uint32_t)(pbeg[u] + c * CH) * 4u : STG_OOB;
            k[u] = __builtin_amdgcn_raw_buffer_load_b32(rc, off, 0, 0);
        }
    };
    auto gather = [&](int c, const int (&k)[S::GPT], i32x4 (&gg)[S::GPT], T &v) {
#pragma unroll
        for (int u = 0; u < S::GPT; ++u) {
            const uint32_t off = c * CH < plen[u] ? (uint32_t)k[u] * rowb + qoff : STG_OOB;
            gg[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0);
        }
        const uint32_t voff = c * CH < vlen ? (uint32_t)(vbeg + c * CH) * (uint32_t)sizeof(T) : STG_OOB;
        if constexpr (sizeof(T) == 8) {
            const i32x2 r = __builtin_amdgcn_raw_buffer_load_b64(rv, voff, 0, 0);
            __builtin_memcpy(&v, &r, 8);
        } else {
            const int32_t r = __builtin_amdgcn_raw_buffer_load_b32(rv, voff, 0, 0);
            __builtin_memcpy(&v, &r, 4);
        }
    };
    auto stash = [&](int buf, const i32x4 (&gg)[S::GPT], T v) {
#pragma unroll
        for (int u = 0; u < S::GPT; ++u) reinterpret_cast<i32x4 *>(s_b[buf])[tid + WG * u] = gg[u];
        s_v[buf][tid] = v;      // every lane (a lane-conditional store leaves its load's wait on some paths only)
    };

    // consumer: row slot s of this lane, its VC columns
    const int wave = tid >> 6, lane = tid & 63;
    const int slot = wave * S::RW + lane / S::CL;
    const int kcol = (lane % S::CL) * S::VC;
    const bool act = slot < R;
    const int my_len = act ? s_len[slot] : 0;
    const int my_row = act ? slot_tab[b * R + slot].x : -1;
    V acc = vzero<T, S::VC>();
    auto fold = [&](int c, int buf) {
        int n = my_len - c * CH;
        n = n < CH ? n : CH;
        const char *bp = s_b[buf] + (size_t)(slot * CH) * SB + kcol * sizeof(T);
        const T *vp = s_v[buf] + slot * CH;
        int j = 0;
        for (; j + STG_FU <= n; j += STG_FU) {
            V bv[STG_FU];
            T av[STG_FU];
#pragma unroll
            for (int q = 0; q < STG_FU; ++q) bv[q] = *reinterpret_cast<const V *>(bp + (j + q) * SB), av[q] = vp[j + q];
#pragma unroll
            for (int q = 0; q < STG_FU; ++q) vfma(acc, av[q], bv[q]);
        }
        for (; j < n; ++j) vfma(acc, vp[j], *reinterpret_cast<const V *>(bp + j * SB));
    };

    // prologue in the steady state's issue order (columns of chunk x + 2 just before the gathers of chunk x):
    // cols 0, 1, then [cols x+2, gathers x] for x < STG_D; chunk 0 -> LDS buffer 0
    load_cols(0, kc[0]);
    load_cols(1, kc[1]);
#pragma unroll
    for (int x = 0; x < STG_D; ++x) {
        load_cols(x + 2, kc[(x + 2) % 3]);
        gather(x, kc[x % 3], g[x], va[x]);
    }
    stash(0, g[0], va[0]);
    __syncthreads();
    // step c (M = c mod STG_UN, every ring index static): columns of chunk c+D+2, gathers of chunk c+D, fold chunk c
    // from LDS buffer c&1, chunk c+1's gathers -> LDS buffer (c+1)&1, barrier
    auto step = [&](int c, auto mc) {
        constexpr int M = decltype(mc)::value;
        load_cols(c + STG_D + 2, kc[(M + STG_D + 2) % 3]);
        gather(c + STG_D, kc[(M + STG_D) % 3], g[M % STG_D], va[M % STG_D]);
        fold(c, M & 1);
        stash((M + 1) & 1, g[(M + 1) % STG_D], va[(M + 1) % STG_D]);
        __syncthreads();
    };
    // whole rounds of STG_UN steps in the loop (its one back edge sees one pending-load state), the rest after it
    int c = 0;
    for (; c + STG_UN <= nch; c += STG_UN) {
        step(c, std::integral_constant<int, 0>());
        step(c + 1, std::integral_constant<int, 1>());
        step(c + 2, std::integral_constant<int, 2>());
        step(c + 3, std::integral_constant<int, 3>());
        step(c + 4, std::integral_constant<int, 4>());
        step(c + 5, std::integral_constant<int, 5>());
    }
    if (c < nch) step(c, std::integral_constant<int, 0>());
    if (c + 1 < nch) step(c + 1, std::integral_constant<int, 1>());
    if (c + 2 < nch) step(c + 2, std::integral_constant<int, 2>());
    if (c + 3 < nch) step(c + 3, std::integral_constant<int, 3>());
    if (c + 4 < nch) step(c + 4, std::integral_constant<int, 4>());
    if (my_row >= 0) vstore<T, S::VC, NTC>(C + (size_t)my_row * ld + kcol, acc);
}

}  // namespace spmm
