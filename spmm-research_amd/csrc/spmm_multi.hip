// spmm_multi.hip -- multi-GPU handles of the C ABI (include/spmm_hip.h: spmm_hip_create_multi), SURVEY §8b/§8e.
//
// The reference harness makes ONE plugin object per run (csr_to_format, spmv_bench.cpp:996) and calls its spmm
// (spmv_bench.cpp:318,372) from one thread; §8b puts the multi-GPU fan-out inside that call.  A multi handle is one
// spmm_hip_t whose rows are split into `ngpus` contiguous nnz-balanced ranges by the reference partitioner
// (loop_partitioner_balance_prefix_sums, lib/parallel_util.h:141-165 == spmm_hip_partition_rows); each range is an
// ordinary single-device child handle (its own copy of its rows of A, its own inspector plan, stream and buffers) on
// its GPU.  One process drives all of them:
//   B    lands on the ROOT device (shard 0's) -- uploaded there (host x) or handed over there (device d_b) -- and is
//        replicated to every other shard's device: root -> peer hipMemcpyPeerAsync over xGMI (default), or one RCCL
//        broadcast over the shards' communicator (SPMM_HIP_BCAST=rccl; needs distinct devices, librccl loaded at
//        first use).  B is read-only, so the copies are the only exchange step in the path (§8e).
//   C    each shard computes its rows into its own HBM.  spmm_hip_run gathers them into the host y (one D2H per
//        shard, concurrently); spmm_hip_run_device gathers them into the caller's root-device C (peer copies);
//        spmm_hip_run_sharded leaves them where they are (the timed multi-GPU path; spmm_hip_shard exposes them).
// Shard streams fork from / join back into the caller's stream by events, so a multi run is stream-ordered like a
// single-device one.  Devices may repeat (every shard on device 0 is the single-GPU test mode of this path).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "spmm_handle.hpp"

using namespace spmm_engine;

#define MCHK(expr)                                                                                       \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess)                                                                            \
            return fail(_e == hipErrorOutOfMemory ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP,                \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                              \
    } while (0)

namespace spmm_engine {

// RCCL entry points, resolved from librccl.so at the first RCCL-mode create (the engine does not link RCCL, so a
// process that never asks for it -- or that already carries PyTorch's own RCCL -- loads no second copy).
struct Rccl {
    void *lib = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclBroadcast) bcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
};
Rccl g_rccl;

int rccl_load() {
    if (g_rccl.lib) return SPMM_HIP_OK;
    void *l = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!l) l = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!l) return fail(SPMM_HIP_ERR_HIP, std::string("SPMM_HIP_BCAST=rccl: cannot load librccl: ") + dlerror());
    Rccl r;
    r.lib = l;
    r.init_all = (decltype(r.init_all))dlsym(l, "ncclCommInitAll");
    r.destroy = (decltype(r.destroy))dlsym(l, "ncclCommDestroy");
    r.bcast = (decltype(r.bcast))dlsym(l, "ncclBroadcast");
    r.group_start = (decltype(r.group_start))dlsym(l, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(l, "ncclGroupEnd");
    r.err = (decltype(r.err))dlsym(l, "ncclGetErrorString");
    if (!r.init_all || !r.destroy || !r.bcast || !r.group_start || !r.group_end || !r.err)
        return fail(SPMM_HIP_ERR_HIP, "librccl lacks ncclCommInitAll / ncclBroadcast / ncclGroupStart / ...");
    g_rccl = r;
    return SPMM_HIP_OK;
}

#define NCHK(expr)                                                                                       \
    do {                                                                                                 \
        ncclResult_t _r = (expr);                                                                        \
        if (_r != ncclSuccess) return fail(SPMM_HIP_ERR_HIP, std::string(#expr) + ": " + g_rccl.err(_r)); \
    } while (0)

struct MultiState {
    std::vector<spmm_hip_t *> shard;     // one child handle per GPU; shard g owns C rows [r0[g], r0[g+1])
    std::vector<int64_t> r0;
    std::vector<int> dev;
    std::vector<hipEvent_t> ev_kern;     // per shard (created on its device): its SpMM is done
    std::vector<hipEvent_t> ev_done;     // per shard: its SpMM and its C hand-back are done
    hipEvent_t ev_fork = nullptr;        // root device: B is ready on the root (shards may start)
    int bcast = SPMM_HIP_BCAST_PEER;
    std::vector<ncclComm_t> comms;       // RCCL mode: one communicator rank per shard
};

namespace {

size_t b_bytes_of(const spmm_hip_t *h, int k) { return (size_t)std::max<int64_t>(h->ncols, 1) * k * h->vsize; }

// Replicate the root-device row-major B at `src` into every shard's B buffer (shard 0 reads src itself when src is
// not its own buffer: then *b0 = src), on the shard streams after the root stream reaches ev_fork.
int broadcast(spmm_hip_t *h, const void *src, int k, hipStream_t root, const void **b0) {
    MultiState &M = *h->multi;
    const size_t bytes = b_bytes_of(h, k);
    MCHK(hipSetDevice(M.dev[0]));
    MCHK(hipEventRecord(M.ev_fork, root));
    *b0 = src;
    if (M.bcast == SPMM_HIP_BCAST_RCCL) {
        for (size_t g = 0; g < M.shard.size(); ++g) {
            MCHK(hipSetDevice(M.dev[g]));
            MCHK(hipStreamWaitEvent(M.shard[g]->stream, M.ev_fork, 0));
        }
        *b0 = M.shard[0]->d_b;
        NCHK(g_rccl.group_start());
        for (size_t g = 0; g < M.shard.size(); ++g)
            NCHK(g_rccl.bcast(g == 0 ? src : M.shard[g]->d_b, M.shard[g]->d_b, bytes, ncclUint8, 0, M.comms[g],
                              M.shard[g]->stream));
        NCHK(g_rccl.group_end());
        return SPMM_HIP_OK;
    }
    for (size_t g = 0; g < M.shard.size(); ++g) {
        MCHK(hipSetDevice(M.dev[g]));
        MCHK(hipStreamWaitEvent(M.shard[g]->stream, M.ev_fork, 0));
        if (g == 0) continue;
        MCHK(hipMemcpyPeerAsync(M.shard[g]->d_b, M.dev[g], src, M.dev[0], bytes, M.shard[g]->stream));
    }
    return SPMM_HIP_OK;
}

// Every shard's SpMM from its replicated B into dst[g] (its own C buffer, or a root-device C at its row offset).
int compute(spmm_hip_t *h, const void *b0, int k, const std::vector<void *> &dst) {
    MultiState &M = *h->multi;
    for (size_t g = 0; g < M.shard.size(); ++g) {
        spmm_hip_t *c = M.shard[g];
        if (c->m == 0) {
            MCHK(hipSetDevice(M.dev[g]));
            MCHK(hipEventRecord(M.ev_kern[g], c->stream));
            continue;
        }
        const void *B = g == 0 ? b0 : c->d_b;
        int st = spmm_hip_run_device(c, B, SPMM_HIP_B_ROW_MAJOR, dst[g], k, c->stream);
        if (st != SPMM_HIP_OK) return st;
        MCHK(hipSetDevice(M.dev[g]));
        MCHK(hipEventRecord(M.ev_kern[g], c->stream));
    }
    return SPMM_HIP_OK;
}

// The caller's stream waits for every shard (events of `which`).
int join(spmm_hip_t *h, hipStream_t root, const std::vector<hipEvent_t> &which) {
    MultiState &M = *h->multi;
    MCHK(hipSetDevice(M.dev[0]));
    for (hipEvent_t e : which) MCHK(hipStreamWaitEvent(root, e, 0));
    return SPMM_HIP_OK;
}

// B on the root device in `layout` -> the root's row-major source (transposed into shard 0's buffer if needed).
int root_source(spmm_hip_t *h, const void *d_b, int layout, int k, hipStream_t root, const void **src) {
    MultiState &M = *h->multi;
    *src = d_b;
    if (layout == SPMM_HIP_B_COL_MAJOR) {
        MCHK(hipSetDevice(M.dev[0]));
        int st = launch_transpose(M.shard[0], d_b, M.shard[0]->d_b, k, root);
        if (st != SPMM_HIP_OK) return st;
        *src = M.shard[0]->d_b;
        M.shard[0]->last_x = nullptr;
    }
    return SPMM_HIP_OK;
}

}  // namespace

int multi_plan(spmm_hip_t *h, int k) {
    MultiState &M = *h->multi;
    if (h->plan.k == k) return SPMM_HIP_OK;
    for (size_t g = 0; g < M.shard.size(); ++g) {
        spmm_hip_t *c = M.shard[g];
        int st = spmm_hip_plan(c, k);
        if (st != SPMM_HIP_OK) return st;
        // every shard receives B and keeps its C rows in its own buffers; the root also stages host x
        if ((st = ensure_buffers(c, true, g == 0, true))) return st;
    }
    Plan pl;
    pl.k = k;
    pl.seq_max = INT32_MAX;
    h->exact.assign((size_t)h->m, 0);
    for (size_t g = 0; g < M.shard.size(); ++g) {
        const spmm_hip_t *c = M.shard[g];
        if (c->m > 0) std::memcpy(h->exact.data() + M.r0[g], c->exact.data(), (size_t)c->m);
        pl.seq_max = std::min(pl.seq_max, c->plan.seq_max);
        pl.exact_rows += c->plan.exact_rows;
        pl.ntile += c->plan.ntile;
        pl.tile_rows += c->plan.tile_rows;
        pl.tile_nnz += c->plan.tile_nnz;
        pl.tile_chunks += c->plan.tile_chunks;
        pl.nseg += c->plan.nseg;
        pl.nwin = std::max(pl.nwin, c->plan.nwin);
        pl.lmax = std::max(pl.lmax, c->plan.lmax);
    }
    const Plan &p0 = M.shard[0]->plan;
    pl.kw = p0.kw, pl.npanels = p0.npanels, pl.cap = p0.cap, pl.win_cols = p0.win_cols, pl.xcd = p0.xcd;
    h->plan = pl;
    h->b_bytes = b_bytes_of(h, k);
    h->c_bytes = (size_t)std::max<int64_t>(h->m, 1) * k * h->vsize;
    return SPMM_HIP_OK;
}

// spmm_hip_run / spmm_hip_run_rowmajor: host x (column-major [k][ncols], or row-major [ncols][k]) -> root ->
// every shard; host y row-major [m][k] gathered shard by shard.  Synchronous.
int multi_run_host(spmm_hip_t *h, const void *x, void *y, int k, bool x_rowmajor) {
    MultiState &M = *h->multi;
    int st = multi_plan(h, k);
    if (st != SPMM_HIP_OK) return st;
    spmm_hip_t *c0 = M.shard[0];
    hipStream_t s = h->stream;                       // the multi handle's own stream, on the root device
    const size_t bytes = b_bytes_of(h, k);
    MCHK(hipSetDevice(M.dev[0]));
    MCHK(hipEventRecord(h->ev[4], s));
    if (h->ncols > 0)
        MCHK(hipMemcpyAsync(x_rowmajor ? c0->d_b : c0->d_xcol, x, (size_t)h->ncols * k * h->vsize,
                            hipMemcpyHostToDevice, s));
    MCHK(hipEventRecord(h->ev[5], s));
    MCHK(hipEventRecord(h->ev[2], s));
    if (!x_rowmajor) {
        st = launch_transpose(c0, c0->d_xcol, c0->d_b, k, s);
        if (st != SPMM_HIP_OK) return st;
    }
    c0->last_x = nullptr;
    MCHK(hipEventRecord(h->ev[3], s));
    MCHK(hipEventRecord(h->ev[0], s));
    const void *b0 = nullptr;
    (void)bytes;
    if ((st = broadcast(h, c0->d_b, k, s, &b0))) return st;
    std::vector<void *> dst(M.shard.size());
    for (size_t g = 0; g < M.shard.size(); ++g) dst[g] = M.shard[g]->d_c;
    if ((st = compute(h, b0, k, dst))) return st;
    if ((st = join(h, s, M.ev_kern))) return st;
    MCHK(hipEventRecord(h->ev[1], s));
    for (size_t g = 0; g < M.shard.size(); ++g) {
        spmm_hip_t *c = M.shard[g];
        MCHK(hipSetDevice(M.dev[g]));
        if (c->m > 0)
            MCHK(hipMemcpyAsync((char *)y + (size_t)M.r0[g] * k * h->vsize, c->d_c, (size_t)c->m * k * h->vsize,
                                hipMemcpyDeviceToHost, c->stream));
        MCHK(hipEventRecord(M.ev_done[g], c->stream));
    }
    if ((st = join(h, s, M.ev_done))) return st;
    MCHK(hipEventRecord(h->ev[6], s));
    MCHK(hipStreamSynchronize(s));
    h->have_times = h->have_copies = true;
    h->have_transpose = !x_rowmajor;
    return SPMM_HIP_OK;
}

// spmm_hip_run_device: d_b on the root device (either layout), d_c on the root device [m][k]; shard 0 writes its
// rows of d_c directly, the others compute in their own HBM and are copied in by peer copies.  Stream-ordered.
int multi_run_device(spmm_hip_t *h, const void *d_b, int layout, void *d_c, int k, hipStream_t s) {
    MultiState &M = *h->multi;
    int st = multi_plan(h, k);
    if (st != SPMM_HIP_OK) return st;
    const bool ev = h->rec_events;
    MCHK(hipSetDevice(M.dev[0]));
    if (ev) MCHK(hipEventRecord(h->ev[0], s));
    const void *src = nullptr, *b0 = nullptr;
    if ((st = root_source(h, d_b, layout, k, s, &src))) return st;
    if ((st = broadcast(h, src, k, s, &b0))) return st;
    std::vector<void *> dst(M.shard.size());
    for (size_t g = 0; g < M.shard.size(); ++g) dst[g] = g == 0 ? d_c : M.shard[g]->d_c;
    if ((st = compute(h, b0, k, dst))) return st;
    for (size_t g = 0; g < M.shard.size(); ++g) {
        spmm_hip_t *c = M.shard[g];
        MCHK(hipSetDevice(M.dev[g]));
        if (g > 0 && c->m > 0)
            MCHK(hipMemcpyPeerAsync((char *)d_c + (size_t)M.r0[g] * k * h->vsize, M.dev[0], c->d_c, M.dev[g],
                                    (size_t)c->m * k * h->vsize, c->stream));
        MCHK(hipEventRecord(M.ev_done[g], c->stream));
    }
    if ((st = join(h, s, M.ev_done))) return st;
    if (ev) MCHK(hipEventRecord(h->ev[1], s));
    h->have_times = ev;
    h->have_transpose = h->have_copies = false;
    return SPMM_HIP_OK;
}

int multi_update_values(spmm_hip_t *h, const void *vals, bool device, hipStream_t s) {
    MultiState &M = *h->multi;
    if (device)
        for (int d : M.dev)
            if (d != M.dev[0])
                return fail(SPMM_HIP_ERR_ARG, "update_values_device on a handle spanning several GPUs: use "
                                              "spmm_hip_update_values (host values, scattered to the shards)");
    for (size_t g = 0; g < M.shard.size(); ++g) {
        spmm_hip_t *c = M.shard[g];
        const char *v = (const char *)vals + (size_t)h->h_row_ptr[(size_t)M.r0[g]] * h->vsize;
        int st = device ? spmm_hip_update_values_device(c, v, s) : spmm_hip_update_values(c, v);
        if (st != SPMM_HIP_OK) return st;
    }
    return SPMM_HIP_OK;
}

int multi_last_times(spmm_hip_t *h, double *out_ms) {
    for (int i = 0; i < 4; ++i) out_ms[i] = 0.0;
    if (!h->have_times) return SPMM_HIP_OK;
    float ms = 0.f;
    MCHK(hipSetDevice(h->multi->dev[0]));
    MCHK(hipEventSynchronize(h->ev[1]));
    MCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    out_ms[0] = ms;                                   // broadcast + every shard's SpMM (the multi-GPU kernel span)
    if (h->have_transpose) {
        MCHK(hipEventElapsedTime(&ms, h->ev[2], h->ev[3]));
        out_ms[1] = ms;
    }
    if (h->have_copies) {
        MCHK(hipEventSynchronize(h->ev[6]));
        MCHK(hipEventElapsedTime(&ms, h->ev[4], h->ev[5]));
        out_ms[2] = ms;
        MCHK(hipEventElapsedTime(&ms, h->ev[1], h->ev[6]));
        out_ms[3] = ms;
    }
    return SPMM_HIP_OK;
}

void multi_info(const spmm_hip_t *h, int64_t *out) {
    const MultiState &M = *h->multi;
    int64_t blocks = 0, split = 0, bytes = 0, fuse = 0;
    for (const spmm_hip_t *c : M.shard) {
        int64_t o[SPMM_HIP_INFO_SLOTS];
        spmm_hip_info(c, o);
        blocks += o[5], split += o[6], bytes += o[7], fuse |= o[18];
    }
    out[5] = blocks;
    out[6] = split;
    out[7] = bytes;
    out[18] = fuse;
}

// The tile kernel the shards run: 2 when any shard runs matrix-core tiles, else 1 when any runs LDS tiles, else 0.
int multi_tile_mode(const spmm_hip_t *h) {
    int mode = 0;
    for (const spmm_hip_t *c : h->multi->shard) mode = std::max(mode, spmm_hip_tile_mode(c));
    return mode;
}

void multi_destroy(spmm_hip_t *h) {
    MultiState *M = h->multi;
    if (!M) return;
    for (size_t g = 0; g < M->shard.size(); ++g) {
        (void)hipSetDevice(M->dev[g]);
        if (M->shard[g] && M->shard[g]->stream) (void)hipStreamSynchronize(M->shard[g]->stream);
        if (g < M->ev_kern.size() && M->ev_kern[g]) (void)hipEventDestroy(M->ev_kern[g]);
        if (g < M->ev_done.size() && M->ev_done[g]) (void)hipEventDestroy(M->ev_done[g]);
    }
    for (ncclComm_t c : M->comms)
        if (c) (void)g_rccl.destroy(c);
    for (spmm_hip_t *c : M->shard) spmm_hip_destroy(c);
    if (!M->dev.empty()) (void)hipSetDevice(M->dev[0]);
    if (M->ev_fork) (void)hipEventDestroy(M->ev_fork);
    delete M;
    h->multi = nullptr;
}

}  // namespace spmm_engine

extern "C" {

int spmm_hip_create_multi(const int32_t *row_ptr, const int32_t *col_idx, const void *values, int64_t m,
                          int64_t ncols, int64_t nnz, int32_t k, int32_t dtype, int32_t ngpus, const int32_t *devices,
                          spmm_hip_t **out) {
    if (!out) return fail(SPMM_HIP_ERR_ARG, "create_multi: out is NULL");
    *out = nullptr;
    if (ngpus < 1 || ngpus > 64) return fail(SPMM_HIP_ERR_ARG, "create_multi: ngpus must be in [1, 64]");
    if (m < 1 || ncols < 0 || nnz < 0 || k < 0 || !row_ptr || (nnz > 0 && (!col_idx || !values)))
        return fail(SPMM_HIP_ERR_ARG, "create_multi: bad CSR arguments");
    if (dtype != SPMM_HIP_F64 && dtype != SPMM_HIP_F32) return fail(SPMM_HIP_ERR_ARG, "create_multi: dtype");
    if (m >= INT32_MAX || ncols >= INT32_MAX || nnz >= INT32_MAX - 4096)
        return fail(SPMM_HIP_ERR_OVERFLOW, "m, ncols and nnz must fit int32 (reference INT_T = int32_t)");
    if (row_ptr[0] != 0 || row_ptr[m] != nnz) return fail(SPMM_HIP_ERR_CSR, "row_ptr[0] != 0 or row_ptr[m] != nnz");
    for (int64_t i = 0; i < m; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return fail(SPMM_HIP_ERR_CSR, "row_ptr not monotone at row " + std::to_string(i));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SPMM_HIP_ERR_NODEVICE, "no HIP device");
    std::vector<int> dev((size_t)ngpus);
    for (int g = 0; g < ngpus; ++g) {
        dev[(size_t)g] = devices ? devices[g] : g;
        if (dev[(size_t)g] < 0 || dev[(size_t)g] >= ndev)
            return fail(SPMM_HIP_ERR_NODEVICE, "create_multi: device index out of range");
    }
    const char *bm = getenv("SPMM_HIP_BCAST");
    const int bcast = (bm && std::strcmp(bm, "rccl") == 0) ? SPMM_HIP_BCAST_RCCL : SPMM_HIP_BCAST_PEER;
    if (bcast == SPMM_HIP_BCAST_RCCL) {
        std::vector<int> sd = dev;
        std::sort(sd.begin(), sd.end());
        if (std::adjacent_find(sd.begin(), sd.end()) != sd.end())
            return fail(SPMM_HIP_ERR_ARG, "SPMM_HIP_BCAST=rccl needs distinct devices (one RCCL rank per GPU)");
        if (int st = rccl_load()) return st;
    }

    spmm_hip_t *h = new spmm_hip_t();
    h->multi = new MultiState();
    MultiState &M = *h->multi;
    M.dev = dev;
    M.bcast = bcast;
    h->device = dev[0];
    h->dtype = dtype;
    h->vsize = dtype == SPMM_HIP_F64 ? 8 : 4;
    h->m = m, h->ncols = ncols, h->nnz = nnz;
    h->h_row_ptr.assign(row_ptr, row_ptr + m + 1);
    auto cleanup = [&](int st) {
        spmm_hip_destroy(h);
        return st;
    };
#define MCHK_C(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess) {                                                                          \
            int _s = (_e == hipErrorOutOfMemory) ? SPMM_HIP_ERR_NOMEM : SPMM_HIP_ERR_HIP;                 \
            fail(_s, std::string(#expr) + ": " + hipGetErrorString(_e));                                 \
            return cleanup(_s);                                                                          \
        }                                                                                                \
    } while (0)
    // shards: the reference partitioner's nnz-balanced contiguous row ranges; A's slices copied to each device
    M.r0.assign((size_t)ngpus + 1, 0);
    for (int g = 0; g < ngpus; ++g) {
        int64_t s = 0, e = 0;
        if (int st = spmm_hip_partition_rows(row_ptr, m, nnz, ngpus, g, &s, &e)) return cleanup(st);
        M.r0[(size_t)g] = s;
        M.r0[(size_t)g + 1] = e;
    }
    std::vector<int32_t> rp;
    for (int g = 0; g < ngpus; ++g) {
        const int64_t s = M.r0[(size_t)g], e = M.r0[(size_t)g + 1];
        rp.resize((size_t)(e - s) + 1);
        for (int64_t i = s; i <= e; ++i) rp[(size_t)(i - s)] = row_ptr[i] - row_ptr[s];
        const int64_t j0 = row_ptr[s], nz = (int64_t)row_ptr[e] - j0;
        spmm_hip_t *c = nullptr;
        // a shard with no rows still gets a handle (m = 0: nothing to run) so every g has one
        static const int32_t zero_col = 0;
        static const double zero_val = 0.0;
        int st = spmm_hip_create(rp.data(), nz > 0 ? col_idx + j0 : &zero_col,
                                 nz > 0 ? (const void *)((const char *)values + (size_t)j0 * h->vsize) : &zero_val,
                                 e - s, ncols, nz, k, dtype, dev[(size_t)g], &c);
        if (st != SPMM_HIP_OK) return cleanup(st);
        M.shard.push_back(c);
        h->a_bytes += c->a_bytes;
    }
    // events per shard device; the root keeps its own stream + timing events (spmm_hip_run, last_times)
    M.ev_kern.assign((size_t)ngpus, nullptr);
    M.ev_done.assign((size_t)ngpus, nullptr);
    for (int g = 0; g < ngpus; ++g) {
        MCHK_C(hipSetDevice(dev[(size_t)g]));
        MCHK_C(hipEventCreateWithFlags(&M.ev_kern[(size_t)g], hipEventDisableTiming));
        MCHK_C(hipEventCreateWithFlags(&M.ev_done[(size_t)g], hipEventDisableTiming));
        if (dev[(size_t)g] != dev[0]) {     // xGMI peer access both ways (the copies work without it, staged)
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, dev[(size_t)g], dev[0]) == hipSuccess && can) {
                hipError_t e = hipDeviceEnablePeerAccess(dev[0], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) MCHK_C(e);
                MCHK_C(hipSetDevice(dev[0]));
                e = hipDeviceEnablePeerAccess(dev[(size_t)g], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) MCHK_C(e);
            }
            (void)hipGetLastError();
        }
    }
    MCHK_C(hipSetDevice(dev[0]));
    MCHK_C(hipEventCreateWithFlags(&M.ev_fork, hipEventDisableTiming));
    MCHK_C(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    for (auto &e : h->ev) MCHK_C(hipEventCreate(&e));
    if (bcast == SPMM_HIP_BCAST_RCCL) {
        M.comms.assign((size_t)ngpus, nullptr);
        ncclResult_t r = g_rccl.init_all(M.comms.data(), ngpus, dev.data());
        if (r != ncclSuccess) {
            M.comms.clear();
            fail(SPMM_HIP_ERR_HIP, std::string("ncclCommInitAll: ") + g_rccl.err(r));
            return cleanup(SPMM_HIP_ERR_HIP);
        }
    }
#undef MCHK_C
    if (k > 0) {
        if (int st = multi_plan(h, k)) return cleanup(st);
    }
    *out = h;
    return SPMM_HIP_OK;
}

int spmm_hip_ngpus(const spmm_hip_t *h, int32_t *ngpus, int32_t *bcast_mode) {
    if (!h || !ngpus) return fail(SPMM_HIP_ERR_ARG, "ngpus: bad arguments");
    *ngpus = h->multi ? (int32_t)h->multi->shard.size() : 1;
    if (bcast_mode) *bcast_mode = h->multi ? h->multi->bcast : SPMM_HIP_BCAST_PEER;
    return SPMM_HIP_OK;
}

int spmm_hip_shard(const spmm_hip_t *h, int32_t g, int32_t *device, int64_t *row0, int64_t *row1, void **d_c) {
    if (!h) return fail(SPMM_HIP_ERR_ARG, "shard: handle is NULL");
    if (!h->multi) {
        if (g != 0) return fail(SPMM_HIP_ERR_ARG, "shard: a single-device handle has shard 0 only");
        if (device) *device = h->device;
        if (row0) *row0 = 0;
        if (row1) *row1 = h->m;
        if (d_c) *d_c = h->d_c;
        return SPMM_HIP_OK;
    }
    const MultiState &M = *h->multi;
    if (g < 0 || g >= (int32_t)M.shard.size()) return fail(SPMM_HIP_ERR_ARG, "shard: index out of range");
    if (device) *device = M.dev[(size_t)g];
    if (row0) *row0 = M.r0[(size_t)g];
    if (row1) *row1 = M.r0[(size_t)g + 1];
    if (d_c) *d_c = M.shard[(size_t)g]->d_c;
    return SPMM_HIP_OK;
}

int spmm_hip_broadcast_b(spmm_hip_t *h, const void *d_b, int32_t b_layout, int32_t k, void *stream) {
    if (!h || !h->multi || !d_b || k < 1) return fail(SPMM_HIP_ERR_ARG, "broadcast_b: needs a multi handle and B");
    if (b_layout != SPMM_HIP_B_COL_MAJOR && b_layout != SPMM_HIP_B_ROW_MAJOR)
        return fail(SPMM_HIP_ERR_ARG, "broadcast_b: b_layout");
    int st = multi_plan(h, k);
    if (st != SPMM_HIP_OK) return st;
    MultiState &M = *h->multi;
    hipStream_t s = (hipStream_t)stream;
    const void *src = nullptr, *b0 = nullptr;
    if ((st = root_source(h, d_b, b_layout, k, s, &src))) return st;
    if ((st = broadcast(h, src, k, s, &b0))) return st;
    if (b0 != M.shard[0]->d_b) {      // peer mode with a caller-owned row-major B: shard 0 keeps a copy too
        MCHK(hipSetDevice(M.dev[0]));
        MCHK(hipMemcpyAsync(M.shard[0]->d_b, b0, b_bytes_of(h, k), hipMemcpyDeviceToDevice, M.shard[0]->stream));
    }
    for (size_t g = 0; g < M.shard.size(); ++g) {
        MCHK(hipSetDevice(M.dev[g]));
        MCHK(hipEventRecord(M.ev_done[g], M.shard[g]->stream));
    }
    return join(h, s, M.ev_done);
}

int spmm_hip_run_sharded(spmm_hip_t *h, int32_t k, void *stream) {
    if (!h || !h->multi || k < 1) return fail(SPMM_HIP_ERR_ARG, "run_sharded: needs a multi handle");
    MultiState &M = *h->multi;
    if (h->plan.k != k) return fail(SPMM_HIP_ERR_K, "run_sharded: broadcast B for this k first (spmm_hip_broadcast_b)");
    hipStream_t s = (hipStream_t)stream;
    const bool ev = h->rec_events;
    MCHK(hipSetDevice(M.dev[0]));
    if (ev) MCHK(hipEventRecord(h->ev[0], s));
    MCHK(hipEventRecord(M.ev_fork, s));
    for (size_t g = 0; g < M.shard.size(); ++g) {
        MCHK(hipSetDevice(M.dev[g]));
        MCHK(hipStreamWaitEvent(M.shard[g]->stream, M.ev_fork, 0));
    }
    std::vector<void *> dst(M.shard.size());
    for (size_t g = 0; g < M.shard.size(); ++g) dst[g] = M.shard[g]->d_c;
    int st = compute(h, M.shard[0]->d_b, k, dst);
    if (st != SPMM_HIP_OK) return st;
    if ((st = join(h, s, M.ev_kern))) return st;
    if (ev) MCHK(hipEventRecord(h->ev[1], s));
    h->have_times = ev;
    h->have_transpose = h->have_copies = false;
    return SPMM_HIP_OK;
}

}  // extern "C"
