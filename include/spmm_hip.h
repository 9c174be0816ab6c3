/*
 * spmm_hip.h -- C ABI of the MI355X-native CSR SpMM engine (libspmm_hip.so).
 *
 * Drop-in boundary for the reference's per-format kernel plugin surface
 * (reference: benchmark_code/CPU/AMD/spmv_code_bench/spmv_kernel.h:9-30, plugin spmm_kernel_csr.cpp:21-66).
 * Plain pointers and sizes only; no C++ or torch types.  Every entry point returns an int status
 * (SPMM_HIP_OK = 0, negative on error; spmm_hip_strerror() names it) where the reference returns void and
 * exits on fatal errors (lib/debug.h:117,127) -- the C++ plugin shim converts a negative status into that exit.
 *
 * Layouts:
 *   A    CSR, int32 row_ptr[m+1], int32 col_idx[nnz], values[nnz] (double or float), 0-based, columns sorted
 *        per row as coo_to_csr leaves them (duplicates allowed).
 *   B    the reference passes x = B COLUMN-major: column n at x[n*ncols .. +ncols) (spmm_kernel_csr.cpp:88).
 *        The engine computes on a ROW-major device copy (B[col][K]); host column-major input is transposed on
 *        the device, outside the SpMM kernel.
 *   C    y = C ROW-major: y[i*K + n] (spmm_kernel_csr.cpp:93); every entry is written (0 for empty rows).
 * Numerics: every C entry is deterministic run to run and within 1e-10 relative normwise (fp64) of the exact sum
 * (SURVEY §8a(ii)).  Rows flagged by spmm_hip_exact_rows -- normally all rows with at most T nonzeros -- are one
 * left-to-right fused multiply-add chain from 0 over the row's nonzeros in CSR order: the same bits as the reference
 * kernel built with its own flags on an FMA x86 host.  T (the split length, spmm_hip_info out[8]) is chosen by the
 * inspector per matrix and K (64..2048) so no serial row outlasts the launch; SPMM_HIP_SEQ_MAX=<n> fixes it; longer
 * rows are cut into T-nonzero pieces combined by a fixed tree.  For long rows at small K the inspector may also
 * give one row several lane groups (vector lanes, out[16]); SPMM_HIP_LANES=-1 keeps every row <= T exact.
 */
#ifndef SPMM_HIP_H
#define SPMM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define SPMM_HIP_OK               0
#define SPMM_HIP_ERR_ARG         -1   /* invalid argument (null pointer, negative size, bad enum)           */
#define SPMM_HIP_ERR_NOMEM       -2   /* device or host allocation failed                                   */
#define SPMM_HIP_ERR_HIP         -3   /* a HIP runtime call failed (details: spmm_hip_last_error_detail)     */
#define SPMM_HIP_ERR_NODEVICE    -4   /* no HIP device / device index out of range                          */
#define SPMM_HIP_ERR_K           -5   /* k does not match the k the handle was created for (see create)     */
#define SPMM_HIP_ERR_CSR         -6   /* malformed CSR (row_ptr not monotone, col_idx out of [0, ncols))     */
#define SPMM_HIP_ERR_OVERFLOW    -7   /* sizes exceed the engine's index range                              */

/* value types (reference: -DValueType=double / float, make.sh:98-102) */
#define SPMM_HIP_F64  0
#define SPMM_HIP_F32  1

/* B layouts for the device entry point */
#define SPMM_HIP_B_COL_MAJOR  0   /* reference layout: x[n*ncols + col]                                    */
#define SPMM_HIP_B_ROW_MAJOR  1   /* engine layout:   B[col*K + n]                                         */

/* upper bound of the split length T (the LDS capacity of one workgroup block, in nonzeros) */
#define SPMM_HIP_SEQ_MAX  2048

typedef struct spmm_hip_handle spmm_hip_t;

/* Factory: replaces `struct Matrix_Format *csr_to_format(INT_T *row_ptr, INT_T *col_ind, ValueType *values,
 * long m, long n, long nnz, int k)` (spmv_kernel.h:29, spmm_kernel_csr.cpp:57-66).  Unlike the reference (which
 * wraps the caller's arrays zero-copy and frees them in its destructor), the engine BORROWS the host arrays for
 * the duration of the call only: it validates A, copies it to device `device`, and builds the workgroup block
 * table (nnz-balanced row blocks).  k is the number of B columns the handle is planned for (0 = decide at the
 * first run; any later run with a different k re-plans).  values points to double (SPMM_HIP_F64) or float. */
int spmm_hip_create(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m, int64_t ncols,
                    int64_t nnz, int32_t k, int32_t dtype, int32_t device, spmm_hip_t **out);

/* Execute, host buffers: replaces `Matrix_Format::spmm(ValueType *x, ValueType *y, INT_T k)`
 * (spmv_kernel.h:18, spmm_kernel_csr.cpp:51-54).  x = host B, column-major [k][ncols]; y = host C, row-major
 * [m][k], overwritten.  Synchronous like the reference: uploads x (skipped when the environment variable
 * SPMM_HIP_ASSUME_X_UNCHANGED=1 and x is the pointer of the previous call), transposes it on the device, runs
 * the SpMM kernel, downloads y. */
int spmm_hip_run(spmm_hip_t *h, const void *x, void *y, int32_t k);

/* Execute, device buffers (kernel-only path; graph-capturable: no allocation or synchronisation inside once the
 * handle is planned for this k and layout).  d_b: device B in `b_layout` (COL_MAJOR is transposed into an
 * internal row-major buffer first, as a separate kernel); d_c: device C row-major [m][k].  stream: a hipStream_t
 * (NULL = the null stream).
 * Concurrency: a handle owns per-run device scratch (the transposed B, split-row partial slots and their arrival
 * counters, the matrix-core plans' out-of-range flag of B, keyed by the handle's launch count), so calls on ONE handle must be serialised on ONE stream (as the reference's plugin is not reentrant,
 * SURVEY §8b).  Two runs of the same handle in flight on different streams race on that scratch; use one handle
 * per stream instead.  A COL_MAJOR run overwrites the internal B, so it also invalidates the upload cache of
 * spmm_hip_run (SPMM_HIP_ASSUME_X_UNCHANGED). */
int spmm_hip_run_device(spmm_hip_t *h, const void *d_b, int32_t b_layout, void *d_c, int32_t k, void *stream);

/* Independent SpMMs of `count` DIFFERENT handles (e.g. the pipeline's K/Q/V projections), run concurrently: the
 * first on `stream`, the others on side streams of this device forked from and joined back into `stream` by events
 * (graph-capturable: a capture on `stream` takes the side streams along; the first call on a device creates its
 * side streams and events, so make it before capturing, like the planning run of each handle).  Same arguments per
 * entry as spmm_hip_run_device; every entry computes exactly what spmm_hip_run_device would. */
int spmm_hip_run_device_batch(int32_t count, spmm_hip_t *const *h, const void *const *d_b, const int32_t *b_layout,
                              void *const *d_c, const int32_t *k, void *stream);

/* Execute, host buffers with B ROW-major (x[col*k + n]; the layout the reference pipeline plugin hands MKL's csrmm,
 * pipeline_code_bench/sddmm_taco_naive.cpp:219-249): uploads x into the engine's B directly (no transpose), runs,
 * downloads y (row-major [m][k]).  Synchronous. */
int spmm_hip_run_rowmajor(spmm_hip_t *h, const void *x, void *y, int32_t k);

/* Replace A's values (same pattern): host array (synchronous) or device array (stream-ordered, graph-capturable).
 * The sparse-attention pipeline's final SpMM multiplies by the SDDMM output, which changes every run
 * (pipeline_code_bench/sddmm_bench.cpp:934-936).  Window-major / tile copies of the values are re-gathered. */
int spmm_hip_update_values(spmm_hip_t *h, const void *vals);
int spmm_hip_update_values_device(spmm_hip_t *h, const void *d_vals, void *stream);

/* Plan for k without running: the inspector (lane layout, block capacity, split length T, K panels of 256-byte B
 * rows when B would crowd the Infinity Cache -- SPMM_HIP_PANEL_K=<cols> overrides) and all allocations happen here, not in
 * run_device. */
int spmm_hip_plan(spmm_hip_t *h, int32_t k);

/* Timing of the LAST run on the handle, from HIP events recorded on the run's stream (blocks until the run
 * finished): out_ms[0] = SpMM kernel(s) only, out_ms[1] = B transpose (0 if none), out_ms[2] = H2D of x,
 * out_ms[3] = D2H of y (the last two only for spmm_hip_run).  spmm_hip_run always records them; spmm_hip_run_device
 * only after spmm_hip_set_timing(h, 1) (or with SPMM_HIP_EVENTS=1 at create): an event pair around every launch
 * costs ~7.5 us of stream time per call on MI355X, so back-to-back callers that time the stream
 * themselves leave it off (all zeros are returned then). */
int spmm_hip_last_times(spmm_hip_t *h, double *out_ms);

/* Statistics hook: replaces Matrix_Format::statistics_start (spmv_kernel.h:19, called before the timed loop at
 * spmv_bench.cpp:350-352): on != 0 makes spmm_hip_run_device record the events spmm_hip_last_times reads. */
int spmm_hip_set_timing(spmm_hip_t *h, int32_t on);

/* Statistics: replaces statistics_print_labels / Matrix_Format::statistics_print_data
 * (spmv_kernel.h:20,30; spmv_bench.cpp:441-443,474-476).  Appends CSV columns to buf (at most buf_n bytes incl.
 * NUL) and returns the number of characters written (<0 on error).  Columns:
 *   kernel_ms,transpose_ms,h2d_ms,d2h_ms,bytes_alg,hbm_gbs_alg,roofline_frac,blocks,split_rows,seq_max,panels,
 *   windows,device,ngpus   (roofline_frac per GPU: hbm_gbs_alg / ngpus / 8000) */
int spmm_hip_stats_labels(char *buf, long buf_n);
int spmm_hip_stats(spmm_hip_t *h, char *buf, long buf_n);

#define SPMM_HIP_INFO_SLOTS 20

/* Properties of the handle (out has SPMM_HIP_INFO_SLOTS = 20 slots): out[0]=m, out[1]=ncols, out[2]=nnz,
 * out[3]=k planned, out[4]=dtype, out[5]=workgroup blocks, out[6]=split rows, out[7]=device bytes held,
 * out[8]=split length T (rows with <= T nonzeros are bit-exact), out[9]=block capacity, out[10]=K-panel width,
 * out[11]=K panels, out[12]=column windows (1 = none; > 1: one launch per window, each row's FMA chain continued
 * through C from window to window, still bit-exact -- SPMM_HIP_WIN_BYTES=<bytes of B per window> forces them,
 * -1 disables), out[13]=window width in columns (0 = none), out[14]=virtual rows (row segments) over all windows,
 * out[15]=1 when workgroup blocks run in XCD-contiguous order (each XCD sweeps one eighth of the rows, so its L2
 * holds only their B rows; SPMM_HIP_XCD=1 forces it, -1 disables it), out[16]=vector lanes: the most row groups one
 * row may get (1 = one group per row; > 1 for long rows at small K, where a block holds fewer rows than groups: the
 * row's nonzeros are dealt round-robin over L groups and the L partials added by a fixed tree -- deterministic,
 * within the 1e-10 normwise contract, not the single chain; SPMM_HIP_LANES=<n> / -1 force / disable),
 * out[17]=C rows computed as one left-to-right FMA chain (bit-identical to the reference; spmm_hip_exact_rows),
 * out[18]=1 when split rows are combined inside the row kernel (the block storing a row's last partial sums it:
 * no combine launch; SPMM_HIP_FUSE=0 keeps the separate combine kernel), out[19]=LDS B tiles (0 = none; see
 * spmm_hip_tile_info). */
int spmm_hip_info(const spmm_hip_t *h, int64_t *out);

/* LDS B tiles of the current plan: runs of up to 64 consecutive rows whose union of columns is
 * read several times (similar or dense rows) are computed by a second kernel that stages each B row of the union
 * in LDS once; every tile row is still one left-to-right FMA chain in CSR order (exact).  out has 7 slots:
 * out[0]=tiles, out[1]=rows in tiles, out[2]=nonzeros in tiles, out[3]=chunks (LDS fills), out[4]=the sampled
 * mean reuse (nonzeros per union column) x 1000 the policy decided on, out[5]=1 when tiles run in XCD order,
 * out[6]=the tile kernel's compute-lane width in 16-byte pieces of a B row (1, 2, 4; SPMM_HIP_TILE_WIDE=<S>).
 * SPMM_HIP_TILES=-1 disables tiles, =1 takes every eligible tile; SPMM_HIP_TILE_REUSE=<x> sets the threshold. */
int spmm_hip_tile_info(const spmm_hip_t *h, int64_t *out);
/* Which kernel runs the tiles of the current plan: 0 = no tiles, 1 = the sparse LDS tile kernel (spmm_tile_kernel),
 * 2 = matrix-core tiles (spmm_mfma_tile_kernel, DESIGN.md §3.9: fp64 32-column panels, 16-row tiles multiplied as
 * dense panels by v_mfma_f64_16x16x4_f64 -- the f64 MFMA is a chain of fused multiply-adds in k order, so these rows
 * are exact too).  SPMM_HIP_MFMA=-1 keeps the sparse tile kernel, 1 takes every eligible 16-row tile. */
int spmm_hip_tile_mode(const spmm_hip_t *h);

/* Which C rows of the current plan are computed as ONE left-to-right FMA chain over the row in CSR order -- the
 * reference kernel's exact operation sequence, so bit-identical to it (mask[i] = 1); the others (rows longer than
 * the split length T, rows given vector lanes) are deterministic and within 1e-10 normwise.  mask has m bytes. */
int spmm_hip_exact_rows(const spmm_hip_t *h, uint8_t *mask);
/* Device buffers owned by the handle (for callers that stage B/C themselves), row-major B of the planned k. */
int spmm_hip_device_ptrs(spmm_hip_t *h, void **d_b_rowmajor, void **d_c);

int spmm_hip_destroy(spmm_hip_t *h);

/* ---- Multi-GPU handles (`ngpus` in the factory, the multi-GPU fan-out inside run; §8e).
 * Same factory arguments as spmm_hip_create plus ngpus and the device of every shard (devices = NULL: 0..ngpus-1;
 * indices may repeat -- every shard on device 0 is the single-GPU test mode).  A's rows are split into ngpus
 * contiguous nnz-balanced ranges by the reference partitioner (spmm_hip_partition_rows =
 * loop_partitioner_balance_prefix_sums, lib/parallel_util.h:141-165); each range becomes a single-device handle on
 * its GPU (own copy of its rows, own inspector plan, stream and buffers).  The handle works with every entry point
 * above except spmm_hip_run_device_batch and spmm_hip_device_ptrs:
 *   spmm_hip_run / spmm_hip_run_rowmajor  host x -> root device (shard 0's) -> replicated to every shard (root->peer
 *       hipMemcpyPeerAsync over xGMI; SPMM_HIP_BCAST=rccl: one RCCL broadcast, distinct devices only) -> every
 *       shard's SpMM concurrently -> its rows of y copied back; synchronous, y identical in layout to one device.
 *   spmm_hip_run_device  d_b and d_c on the ROOT device; shard 0 writes its rows of d_c in place, the others are
 *       copied in (peer copies); stream-ordered on `stream` (shard streams fork/join by events).
 *   spmm_hip_update_values  host values, scattered to the shards (the device variant only when all shards share
 *       one device).
 *   spmm_hip_last_times  out_ms[0] = broadcast + all shards' SpMMs (the multi-GPU kernel span).
 * Results: every shard is an independent plan over its rows, so a row is computed exactly as a one-device handle
 * over those same rows computes it; spmm_hip_exact_rows concatenates the shards' masks. */
#define SPMM_HIP_BCAST_PEER  0   /* B replicated by root -> peer hipMemcpyPeerAsync (default)              */
#define SPMM_HIP_BCAST_RCCL  1   /* B replicated by one RCCL broadcast (SPMM_HIP_BCAST=rccl at create)     */
int spmm_hip_create_multi(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m,
                          int64_t ncols, int64_t nnz, int32_t k, int32_t dtype, int32_t ngpus, const int32_t *devices,
                          spmm_hip_t **out);
/* Shards of a handle (1 for spmm_hip_create handles) and the broadcast mode in use. */
int spmm_hip_ngpus(const spmm_hip_t *h, int32_t *ngpus, int32_t *bcast_mode);
/* Shard g: its device, its C rows [*row0, *row1) and its device-local C buffer ([rows][k], row-major). */
int spmm_hip_shard(const spmm_hip_t *h, int32_t g, int32_t *device, int64_t *row0, int64_t *row1, void **d_c);
/* The timed multi-GPU path: replicate B (root device, either layout) once, then spmm_hip_run_sharded computes every
 * shard's rows into its own C buffer (spmm_hip_shard), leaving C sharded -- no gather inside the loop (§8e). */
int spmm_hip_broadcast_b(spmm_hip_t *h, const void *d_b, int32_t b_layout, int32_t k, void *stream);
int spmm_hip_run_sharded(spmm_hip_t *h, int32_t k, void *stream);

/* nnz-balanced row split (reference: loop_partitioner_balance_prefix_sums, lib/parallel_util.h:141-165, with
 * binary_search lib/macros/macrolib.h:471-524): worker w of W gets rows [*start, *end).  Used for GPU shards. */
int spmm_hip_partition_rows(const int32_t *row_ptr, int64_t m, int64_t nnz, int64_t num_workers,
                            int64_t worker_pos, int64_t *start, int64_t *end);

/* Algorithmic byte model per SpMM call (reference SpMV model spmv_operator.cu:30-32 extended to
 * K columns): 4(m+1) + (4+s)nnz + s*K*ncols + s*K*m, s = sizeof(value). */
double spmm_hip_bytes_alg(int64_t m, int64_t ncols, int64_t nnz, int32_t k, int32_t dtype);

/* Diagnostics (host only, no device needed): the inspector's work decomposition for a CSR pattern, for tests.
 * win_cols = 0: one window (the plain row split); > 0: column windows of that many columns (chained mode; every
 * row's columns must be sorted).  On success the arrays are malloc'ed; release with spmm_hip_debug_free.
 *   vrow_ptr[nv+1]   virtual-row offsets into the (window-major, if windowed) nonzero order
 *   vdest[nv]        destination code (0-length if no row is split and there are no windows): plain split mode
 *                    d (C row >= 0, slot -s-1); windowed mode (d << 1) | continue
 *   blk[2*nblk]      {first, end} virtual rows of each workgroup block
 *   win_blk[nwin+1]  blocks of window w: [win_blk[w], win_blk[w+1])
 *   perm[nz]         windowed mode: original nonzero index of each position (NULL otherwise)
 *   long_rows[4*nlong] {row, first slot, slots, 0} of each split row */
typedef struct {
    int64_t nv, nblk, nwin, nz, nlong, nslots;
    int32_t *vrow_ptr, *vdest, *blk, *win_blk, *long_rows;
    int64_t *perm;
} spmm_hip_inspection_t;
int spmm_hip_debug_inspect(const int32_t *row_ptr, const int32_t *col_idx, int64_t m, int64_t ncols, int32_t T,
                           int32_t cap, int64_t win_cols, spmm_hip_inspection_t *out);
void spmm_hip_debug_free(spmm_hip_inspection_t *ins);

/* Diagnostics (host only): the tile decomposition for a CSR pattern with sorted rows (tests).  Rows of at most T
 * nonzeros are grouped in runs of up to rmax; a run becomes a tile when its reuse is >= min_reuse; its union of
 * columns is cut into chunks of <= uc columns and <= capa entries (incl. padding); a run whose union exceeds colmax
 * columns or that would make more than dmax chunks is halved until it fits (colmax / dmax <= 0: no limit).  Arrays malloc'ed, release with
 * spmm_hip_debug_tiles_free:
 *   tiles[4*ntile]       {first row, rows, first chunk, chunks}
 *   chunks[4*(nchunk+1)] {first tcol, columns, first position, first tseg} (+ sentinel)
 *   tcol[ncol]           union columns, chunk by chunk
 *   tseg[nseg]           per chunk, rows+1 segment starts relative to the chunk's first position (8-aligned);
 *                        every row segment is padded to a multiple of 4 entries
 *   perm[nz], tlidx[nz]  position -> original nonzero (-1 = padding) and chunk-local column (0xFFFF = padding)
 *   in_tile[m]           1 for rows in a tile */
typedef struct {
    int64_t ntile, nchunk, ncol, nseg, nz, m;
    int32_t *tiles, *chunks, *tcol;
    uint16_t *tseg, *tlidx;
    int64_t *perm;
    uint8_t *in_tile;
} spmm_hip_tiles_t;
int spmm_hip_debug_tiles(const int32_t *row_ptr, const int32_t *col_idx, int64_t m, int64_t ncols, int32_t T,
                         int32_t rmax, int32_t uc, int32_t capa, double min_reuse, int32_t colmax, int32_t dmax,
                         spmm_hip_tiles_t *out);
void spmm_hip_debug_tiles_free(spmm_hip_tiles_t *t);


/* Diagnostics (host only): the inspector's decisions for (CSR, k, dtype) without a device -- what spmm_hip_plan would
 * plan (tools/plan_census.py runs it over the whole medium dataset).  mfma: the SPMM_HIP_MFMA override (-1 no
 * matrix-core tiles, 0 policy, 1 every eligible tile, 2 the policy's gate forced open).  gate_only != 0: stop after
 * the matrix-core gate, which reads the columns of its sampled 16-row tiles only (rows t*16 .. t*16+15 for
 * t = i * ceil(m/16) / min(256, ceil(m/16)), i = 0..); col_idx then only needs those rows filled.  out has
 * SPMM_HIP_PLAN_SLOTS doubles: [0] tile mode (0 none, 1 LDS, 2 matrix-core; gate-only: 2 or 0), [1] gate verdict,
 * [2] sampled 16-row reuse, [3] fraction of sampled tiles taken, [4] est. nonzeros in taken tiles, [5] est. chunks,
 * [6] largest sampled chunk count, [7] model time with tiles (us), [8] model time without (us), [9] tiles sampled,
 * [10] split length T, [11] piece length of rows > T, [12] K-panel width, [13] K panels, [14] tiles built,
 * [15] nonzeros in tiles, [16] chunks, [17] row-kernel blocks, [18] split rows, [19] exact rows, [20] vector lanes,
 * [21] XCD order, [22] column windows, [23] 1 = gate only, [24]/[25] plan fingerprint (low / high 32 bits; two
 * plans are the same exactly when these agree), [26] est. taken tiles, [27] paired short rows,
 * [28] the pair policy's sampled reuse of 16-row windows (0 = not sampled), [29] block capacity (nonzeros; 4096 =
 * the wide window). */
#define SPMM_HIP_PLAN_SLOTS 32
int spmm_hip_debug_plan(const int32_t *row_ptr, const int32_t *col_idx, int64_t m, int64_t ncols, int32_t k,
                        int32_t dtype, int32_t mfma, int32_t gate_only, double *out);
/* Diagnostics (host only): the matrix-core gate's cost model on a recorded sample -- sample[7] =
 * {tiles sampled, mean reuse, fraction taken, est. taken tiles, est. nonzeros in them, est. chunks, largest sampled
 * chunk count} as spmm_hip_debug_plan reports them ([9], [2], [3], [26], [4], [5], [6]), kw its K-panel width
 * ([12]), dtype the value type (its constant set); the matrix is taken as square (ncols = m, as every dataset
 * line); out[3] = {verdict, model
 * time with matrix-core tiles (us), without (us)}.  Lets a census re-decide with this library's constants without
 * regenerating the matrices (tools/plan_census.py --regate). */
int spmm_hip_debug_gate(int64_t m, int64_t nnz, int32_t k, int32_t kw, int32_t dtype, const double *sample,
                        double *out);

const char *spmm_hip_strerror(int status);
const char *spmm_hip_last_error_detail(void);
int spmm_hip_device_count(int *count);
const char *spmm_hip_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SPMM_HIP_H */
