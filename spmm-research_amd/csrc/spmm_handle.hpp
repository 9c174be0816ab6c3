// spmm_handle.hpp -- the engine handle (struct spmm_hip_handle behind include/spmm_hip.h) and what the engine's
// translation units share: spmm_engine.hip (single-device engine, inspector, launches) and spmm_multi.hip (multi-GPU
// handles: one child handle per GPU, SURVEY §8b "ngpus").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/spmm_hip.h"

namespace spmm_engine {

extern thread_local std::string g_detail;      // spmm_hip_last_error_detail()
int fail(int status, const std::string &what);  // records the detail, returns status

// Production kernel variant (tools/tune_kernel.py on MI355X).
#ifndef DEF_U
#define DEF_U 16
#endif
#ifndef DEF_NTC
#define DEF_NTC 1
#endif
#ifndef DEF_DMA
#define DEF_DMA 0
#endif
#ifndef DEF_BUF
#define DEF_BUF 1
#endif


struct Plan {
    int k = -1;
    int kw = 0, npanels = 0;   // panel width (columns) and count
    int ygrid = 0;             // 1 = the row kernel runs all panels in one launch (blockIdx.y = panel)
    int seq_max = 0;           // T: rows of <= T nonzeros are one chain (exact)
    int piece = 0;             // rows longer than T are cut into pieces of this many nonzeros (T, or GAP_SEQ_MAX)
    int cap = 0;               // block capacity (nonzeros)
    int block_rows = 512;      // virtual rows per block at most (CAP_ROWS; SPMM_HIP_BLOCK_ROWS lowers it)
    int64_t win_cols = 0;      // column-window width (0 = one window over all columns)
    int nwin = 1;              // column windows (one launch each per K panel)
    int64_t nseg = 0;          // virtual rows (segments) over all windows
    int xcd = 0;               // 1 = XCD-contiguous block order (each XCD sweeps one eighth of the rows)
    int lmax = 1;              // vector lanes: max groups per row (1 = every row one group, exact)
    int pair = 0;              // 1 = paired short rows: two rows of <= U/2 nonzeros per gather batch (exact)
    double pair_reuse = 0.0;   // the pair policy's sampled 16-row-window reuse (0 = not sampled)
    int64_t exact_rows = 0;    // C rows computed as one left-to-right chain (bit-identical to the reference)
    int ntile = 0;             // LDS B tiles (spmm_tile_kernel), rows and nonzeros they cover, their chunks
    int tile_xcd = 0;          // tiles in XCD-contiguous order
    int tile_wide = 1;         // compute-lane width in 16-byte pieces of a B row (1, 2, 4), where RPG allows
    int tile_mfma = 0;         // 1 = the tiles run on the matrix cores (spmm_mfma_tile_kernel, 16-row wave tiles)
    int64_t tile_rows = 0, tile_nnz = 0, tile_chunks = 0;
    double tile_reuse = 0.0;   // sampled mean reuse (nnz per union column) the policy saw
};

struct Variant {
    int u = DEF_U, ntc = DEF_NTC, dma = DEF_DMA, buf = DEF_BUF;
    int seq_max = 0, cap = 0;  // 0 = inspector policy
    int panel_k = 0;           // 0 = inspector policy
    int64_t win_bytes = 0;     // 0 = inspector policy, < 0 = no column windows, > 0 = window of this many B bytes
    int xcd = 0;               // 0 = inspector policy, < 0 = off, > 0 = XCD-contiguous block order
    int lanes = 0;             // 0 = inspector policy, < 0 = off (exact rows), > 0 = vector lanes up to this many
    int tiles = 0;             // 0 = inspector policy, < 0 = off, > 0 = every eligible tile with reuse >= 1
    int mfma = 0;              // 0 = inspector policy, < 0 = sparse LDS tiles only, > 0 = matrix-core tiles when eligible
};

struct MultiState;                              // spmm_multi.hip

// engine internals the multi-GPU layer drives (spmm_engine.hip)
int launch_transpose(spmm_hip_t *h, const void *X, void *Bt, int K, hipStream_t s);
int ensure_buffers(spmm_hip_t *h, bool b, bool xcol, bool c);   // the handle's own B / staging / C, at first use

// multi-GPU handles (spmm_multi.hip); h->multi != nullptr routes the public entry points here
int multi_plan(spmm_hip_t *h, int k);
int multi_run_host(spmm_hip_t *h, const void *x, void *y, int k, bool x_rowmajor);
int multi_run_device(spmm_hip_t *h, const void *d_b, int layout, void *d_c, int k, hipStream_t s);
int multi_update_values(spmm_hip_t *h, const void *vals, bool device, hipStream_t s);
int multi_last_times(spmm_hip_t *h, double *out_ms);
void multi_info(const spmm_hip_t *h, int64_t *out);
int multi_tile_mode(const spmm_hip_t *h);
void multi_destroy(spmm_hip_t *h);

}  // namespace spmm_engine

struct spmm_hip_handle {
    int device = 0;
    int dtype = SPMM_HIP_F64;
    size_t vsize = 8;
    int64_t m = 0, ncols = 0, nnz = 0;
    std::vector<int32_t> h_row_ptr;  // kept for re-inspection at plan time

    int32_t *d_col = nullptr;
    void *d_val = nullptr;

    // inspector output (per plan)
    spmm_engine::Plan plan;
    spmm_engine::Variant var;
    int64_t nv = 0;                  // virtual rows
    int nblk = 0, nlong = 0, nslots = 0;
    int32_t *d_vrow_ptr = nullptr, *d_vdest = nullptr;
    int4 *d_blk = nullptr;           // {first, end | flags, vrow_ptr[first], vrow_ptr[end]} per block
    int4 *d_long_rows = nullptr;
    std::vector<int> win_blk;        // blocks of column window w: [win_blk[w], win_blk[w+1])
    std::vector<int64_t> win_v;      // virtual rows of column window w: [win_v[w], win_v[w+1])
    std::vector<uint8_t> exact;      // per C row: 1 = one left-to-right FMA chain (spmm_hip_exact_rows)
    int32_t *d_lr_cnt = nullptr;     // fused combine: per split row, pieces stored so far in this launch (re-armed to 0)
    int32_t *d_slot_lr = nullptr;    // fused combine: partial slot -> split row
    bool fuse = false;               // split rows combined inside the row kernel (no spmm_combine_kernel launch)
    int32_t *d_wcol = nullptr;       // chained mode: col_idx / values in window-major segment order
    void *d_wval = nullptr;
    int4 *d_tiles = nullptr, *d_tchunk = nullptr;   // tile mode (spmm_tile_kernel / spmm_mfma_tile_kernel)
    int32_t *d_tcol = nullptr;       // union columns (matrix-core tiles: per chunk 48 slots in [g][k step] order)
    uint16_t *d_tseg = nullptr, *d_tlidx = nullptr;  // (matrix-core tiles: d_tlidx = panel cells)
    void *d_tval = nullptr;
    long long *d_tstamps = nullptr;  // SPMM_HIP_TILE_STAMPS=1: per tile {start, end, wait, compute} s_memtime stamps
    int32_t *d_wperm = nullptr;      // window-major position -> nonzero (value updates re-gather wval)
    int32_t *d_tperm = nullptr;      // tile chunk-major position -> nonzero, -1 = padding (value updates re-gather tval)
    int *d_mflag = nullptr;          // matrix-core tiles: {A, B} operand outside the exact range (spmm_mfma.hpp)
    int mflag_seq = 0;               // matrix-core launches so far: mflag[1] == seq marks THIS launch's B as out of range
    int64_t nwperm = 0, ntperm = 0;

    // per-k buffers
    void *d_b = nullptr;      // row-major B [ncols][k]
    void *d_xcol = nullptr;   // column-major staging for host uploads / device col-major input
    void *d_c = nullptr;      // row-major C [m][k]
    void *d_part = nullptr;   // split-row partials [nslots][k]
    size_t b_bytes = 0, c_bytes = 0, insp_bytes = 0;

    const void *last_x = nullptr;
    hipStream_t stream = nullptr;  // own stream for spmm_hip_run
    hipStream_t side = nullptr;    // matrix-core plans: the row kernel's leftover rows run here, beside the tiles
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t ev[8] = {};
    bool have_times = false, have_transpose = false, have_copies = false;
    bool rec_events = false;         // run_device records timing events (spmm_hip_set_timing / SPMM_HIP_EVENTS=1)
    int64_t a_bytes = 0;
    spmm_engine::MultiState *multi = nullptr;   // multi-GPU handle: its shards (nullptr = one device)
};
