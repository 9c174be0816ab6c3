#!/usr/bin/env python3
"""bench.py -- headline benchmark: CSR SpMM C = A*B, K=32, fp64, synthetic matrices, MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  N>1 runs one rank per GPU; when it is not
started by torch.distributed.run (no WORLD_SIZE in the environment) it starts torch.distributed.run itself as a
CHILD process (before anything touches the GPU) and exits with its status.  A world size that differs from --gpus
is an error (exit 2).  One "step" = one SpMM over the rank's row shard, inputs resident in HBM.  Rank 0 prints ONE
JSON line.

The line (default, --workload dataset) measures BASELINE.json's metric on its own workload, "synthetic medium
dataset, CSR SpMM K=32 fp64":
  value     every --dataset-stride-th line of synthetic_matrices_medium_dataset (stride 80 = 203 matrices, K=32
            fp64).  One STEP = one SpMM over every matrix of the sample: per matrix --warmup untimed launches, then
            --steps launches timed by HIP events on the launch stream (a calibrated GPU-side pre-roll keeps host
            enqueue gaps out of the timed region).  ms_per_step = the sum over matrices of the per-launch time;
            value = sum(2*nnz*K) / ms_per_step = the aggregate GFLOP/s; roofline = sum of algorithmic bytes over the
            same time, with the median / p10 / p90 per-matrix fractions, per-matrix PMC traffic when profiles/ holds
            it for this engine build and the gather ceiling; cpu_baseline = the oracle's compute_csr on
            a time-bounded subset of the same matrices (same A and B), whose C also checks the GPU's C bit for bit on
            the rows the engine reports exact.
            At N > 1 (weak scaling: the metric's workload sharded as independent matrices, no collective in the
            data path) rank r runs its own stride-80 sample at offset r*80/N, so every GPU carries a statistically
            equal share; value = the flops of all ranks / the max over ranks of their summed HIP-event time.
  config2   (sub-record, N=1) BASELINE configs[1], SURVEY.md §8d: generator line
            1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14, K=32 fp64; --steps / --warmup launches, its
            own roofline (PMC traffic, gather ceiling), CPU baseline with the oracle check over every row, and the
            plugin end-to-end (PCIe) call.  At N > 1: config 2 weak (every rank a config-2-sized nnz-balanced row range
            of one N-times-larger matrix), plus the in-process multi-GPU handle record.
  config4   (sub-record, N > 1) BASELINE configs[3]: the largest avg-20 skew-10^4 line of
            synthetic_matrices_large_dataset.txt with gamma row lengths (7477550 rows, 150 M nonzeros) split N ways
            with the reference partitioner (strong scaling), B broadcast over RCCL once, max-over-ranks HIP-event
            time, imbalance, C all-gathered once (timed).
Other workloads (as the line itself):
  config2   (N >= 1) the config-2 record above (--scaling strong: the single config-2 matrix split N ways).
  config4   (N >= 1) the config-4 record above.
  medium-sample  the dataset record with --dataset-iters / --dataset-warmup launches per matrix.
  twins     (config 5) the 52 validation twins (reference config.sh:283-339) at K=32, fp64 AND fp32: per dtype
            aggregate GFLOP/s and median fraction, and a cpu_baseline on every twin in the same run (time-bounded).
  pipeline   the sparse-attention pipeline consumer, fp32, n=512 (see run_pipeline).

A values: the generator's seeded U[0.5, 1.5).  B: config 2 / config 4: drand48(seed 42) drawn on the host in the
reference harness's column-major layout [K][ncols] (the x the CPU baseline multiplies), uploaded transposed to the
engine's row-major layout; dataset / twins: torch.rand(seed 42) on the device (copied back column-major for the
CPU baseline).  Everything resident in HBM in the timed region.

Multi-GPU (--scaling, default weak): WEAK = the line's shape N times over (N x rows, N x columns, bw/N: the same
absolute column window) split into N nnz-balanced row ranges with the reference partitioner
loop_partitioner_balance_prefix_sums (lib/parallel_util.h:141-165), so every GPU carries one line's work.  STRONG =
the line's matrix itself split N ways (a fixed global problem).  Each rank generates only its rows; B is broadcast from rank 0 once at setup
(timed); C stays sharded in the timed loop and is all-gathered once afterwards (timed).  --dist-backend gloo (test
mode) lets several ranks share one GPU (collectives staged through host memory).

Self-check (every rank, every run): sampled rows of the rank's C against a numpy recomputation (normwise 1e-10
fp64 / (n+1)*2^-24 fp32); a failure or a non-finite C exits non-zero.  Bit-exact parity against the oracle lives in
tests/ (the oracle is test infrastructure; only the cpu_baseline legs use it).

roofline: algorithmic bytes per launch (4(m+1) + (4+s)nnz + s*K*ncols + s*K*m) over the HIP-event
launch time against 8 TB/s; "traffic" = PMC past-L2 bytes per launch (tools/collect_pmc.py, tools/pmc_dataset.py)
when profiles/ holds them for this engine build; "achievable" = the gather ceiling: that traffic at
the chip's measured random-row gather rate for a table of B's size, and the L2 requests at the L2-resident gather
rate (profiles/r01_gather_probe.jsonl) -- "frac_of_achievable" = ceiling time / measured time.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
# the CPUs this process may use, read before the HIP runtime starts: on the GPU box the runtime narrows the main
# thread's affinity (2 of 256 CPUs were seen), which OpenMP threads started later would inherit
_AFFINITY0 = os.sched_getaffinity(0)

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "GFLOP/s + achieved HBM GB/s, synthetic medium dataset, CSR SpMM K=32 fp64"
# random-row gather rates of this chip by table size (profiles/r01_gather_probe.jsonl: 256-B rows, 16 in flight per
# 16-lane group, all CUs): bytes -> TB/s.  The L2-resident rate bounds the on-chip request path.
GATHER_PROBE = [(2 << 20, 27.79), (16 << 20, 9.62), (64 << 20, 7.50), (160 << 20, 7.09), (256 << 20, 7.19),
                (1 << 30, 6.85), (4 << 30, 5.86)]
L2_GATHER_TBS = 27.79
L2_LINE = 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--workload", choices=["dataset", "config2", "config4", "medium-sample", "twins", "pipeline"],
                    default="dataset")
    ap.add_argument("--pipe-m", type=int, default=512, help="pipeline: weight rows = mask size")
    ap.add_argument("--pipe-k", type=int, default=512, help="pipeline: weight columns (rows of x)")
    ap.add_argument("--pipe-n", type=int, default=512, help="pipeline: columns of x (NUM_COLS)")
    ap.add_argument("--pipe-density", type=float, default=0.3, help="pipeline: weight density (1 - pruning)")
    ap.add_argument("--pipe-mask-density", type=float, default=0.05)
    ap.add_argument("--pipe-band", type=int, default=16)
    ap.add_argument("--pipe-mode", type=int, default=0, help="pipeline: SDDMM flags (0 reference, 1 QK^T, |2 softmax)")
    ap.add_argument("--gen", default=None, help="override: 11-field generator line of the global matrix")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="weak")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: test mode, ranks may share one GPU (collectives staged through host memory)")
    ap.add_argument("--dump-c", default=None, help="rank 0 writes a row sample of the (gathered) C + exact mask (npz)")
    ap.add_argument("--no-multi-handle", action="store_true",
                    help="N>1: skip the in-process multi-GPU handle record (peer vs RCCL B broadcast)")
    ap.add_argument("--no-dataset", action="store_true",
                    help="--workload dataset: skip the dataset pass (sub-records only; tests and PMC tools)")
    ap.add_argument("--no-config2", action="store_true", help="--workload dataset: skip the config-2 sub-record")
    ap.add_argument("--no-config4", action="store_true", help="--workload dataset, N > 1: skip the config-4 sub-record")
    ap.add_argument("--strong-gen", default=None,
                    help="override the config-4 generator line (the strong-split sub-record; tests use a small one)")
    ap.add_argument("--dump-c-strong", default=None, help="rank 0 writes a row sample of the config-4 record's C (npz)")
    ap.add_argument("--dataset-stride", type=int, default=80, help="dataset: every n-th medium-dataset line")
    ap.add_argument("--dataset-out", default=None,
                    help="write the dataset pass's per-matrix records (JSONL; rank r appends .r<r> at N > 1)")
    ap.add_argument("--dataset-offset", type=int, default=0)
    ap.add_argument("--dataset-iters", type=int, default=10, help="dataset / twins: timed launches per matrix")
    ap.add_argument("--dataset-warmup", type=int, default=3)
    ap.add_argument("--dataset-cpu-seconds", type=float, default=20.0, help="dataset: CPU-baseline budget")
    ap.add_argument("--twins-cpu-seconds", type=float, default=1.0, help="twins: CPU-baseline budget per twin/dtype")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-warmup", type=int, default=100, help="CPU-baseline warm-up calls (reference harness: 100)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of timed CPU-baseline calls (the reference's 100 timed calls fit ~9 s on 16 cores)")
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "pmc_latest.json"),
                    help="config-2 per-launch PMC counters (tools/collect_pmc.py)")
    ap.add_argument("--pmc-dataset", default=str(ROOT / "profiles" / "pmc_dataset_latest.json"),
                    help="per-matrix PMC records (tools/pmc_dataset.py), keyed by line, K, dtype and engine build")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """--gpus N without torch.distributed.run: start it as a child process (nothing here has touched the GPU) and
    return its exit status.  Never an exec: the child is a fresh process."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_share() -> tuple[int, str]:
    """Threads for the CPU baseline: the CPUs this process may run on (its affinity at start; restored here for
    this thread, so the OpenMP team the baseline starts can use them), capped by the cgroup CPU quota and by
    OMP_NUM_THREADS when the environment sets it (the GPU box: quota 16 CPUs, OMP_NUM_THREADS=16); and the CPU
    model."""
    try:
        os.sched_setaffinity(0, _AFFINITY0)
    except OSError:
        pass
    n = len(_AFFINITY0)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    model = "unknown CPU"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model


def engine_sha256() -> str:
    """Fingerprint of the engine build: its device/host sources and the Makefile (flags), so PMC numbers collected for
    one engine version stay attached to it across rebuilds (the .so bytes themselves are not reproducible)."""
    import hashlib
    h = hashlib.sha256()
    pkg = ROOT / "spmm-research_amd"
    for f in (pkg / "csrc" / "spmm_engine.hip", pkg / "csrc" / "spmm_kernels.hpp", pkg / "csrc" / "spmm_handle.hpp",
              pkg / "csrc" / "spmm_multi.hip", pkg / "csrc" / "spmm_mfma.hpp", ROOT / "include" / "spmm_hip.h", pkg / "Makefile"):
        h.update(f.read_bytes())
    return h.hexdigest()


def gather_rate_tbs(table_bytes: float) -> float:
    """Measured random-row gather rate (TB/s) for a table of `table_bytes` (log-linear between probe points)."""
    pts = GATHER_PROBE
    if table_bytes <= pts[0][0]:
        return pts[0][1]
    for (b0, r0), (b1, r1) in zip(pts, pts[1:]):
        if table_bytes <= b1:
            f = (math.log(table_bytes) - math.log(b0)) / (math.log(b1) - math.log(b0))
            return r0 + f * (r1 - r0)
    return pts[-1][1]


def achievable(t_ms: float, traffic: float | None, l2_req: float | None, b_bytes: float,
               bytes_alg: float | None = None) -> dict | None:
    """The gather ceiling of a launch: its measured past-L2 bytes at the chip's random-row gather rate
    for a table of B's size, its L2 requests (x 128 B) at the L2-resident gather rate, and (round 6) its compulsory
    algorithmic bytes at the HBM peak; the largest time is the ceiling.  The third term matters where the gather
    terms price streamed bytes at an on-chip rate: at K = 1 the past-L2 bytes are A's once-read stream (1.04x the
    algorithmic bytes), which no launch moves faster than HBM, so without it the "ceiling" sat below the roofline
    time itself.  frac_of_achievable = ceiling / measured (1.0 = at the ceiling)."""
    if traffic is None or t_ms <= 0:
        return None
    r = gather_rate_tbs(b_bytes)
    t_past = traffic / (r * 1e12) * 1e3
    t_l2 = (l2_req * L2_LINE) / (L2_GATHER_TBS * 1e12) * 1e3 if l2_req else 0.0
    t_hbm = bytes_alg / (HBM_PEAK_GBS * 1e9) * 1e3 if bytes_alg else 0.0
    t = max(t_past, t_l2, t_hbm)
    bound = "HBM compulsory" if t == t_hbm and t_hbm > 0 else "past-L2 gather" if t_past >= t_l2 else "L2 requests"
    return {"t_ms": round(t, 5), "bound": bound, "past_l2_gather_tbs": round(r, 2), "t_past_l2_ms": round(t_past, 5),
            "t_l2_ms": round(t_l2, 5), "t_hbm_ms": round(t_hbm, 5), "frac_of_achievable": round(t / t_ms, 4)}


_PREROLL: dict = {}


def preroll(torch, stream, ms: float = 2.0) -> None:
    """GPU-side pre-roll in front of a timed batch: a spin kernel of ~`ms` keeps the stream busy while the host
    enqueues the timed launches, so a host-side stall (the generator thread, the garbage collector) never becomes an
    idle gap between the events.  The events bracket only the launches; the spin rate is calibrated once."""
    try:
        if "cyc_per_ms" not in _PREROLL:
            with torch.cuda.stream(stream):
                torch.cuda._sleep(100_000)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                torch.cuda._sleep(2_000_000)
                e1.record(stream)
            torch.cuda.synchronize()
            _PREROLL["cyc_per_ms"] = 2_000_000 / max(e0.elapsed_time(e1), 1e-3)
        if _PREROLL["cyc_per_ms"]:
            with torch.cuda.stream(stream):
                torch.cuda._sleep(int(ms * _PREROLL["cyc_per_ms"]))
    except Exception:  # no spin kernel in this torch build: time without a pre-roll
        _PREROLL["cyc_per_ms"] = None


def timed_launches(torch, stream, launch, iters: int) -> float:
    """HIP-event time (ms) per launch of `iters` back-to-back launches on `stream`, behind a pre-roll."""
    import gc
    gc.collect()
    gc.disable()
    try:
        preroll(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            launch()
        e1.record(stream)
    finally:
        gc.enable()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / max(iters, 1)


def cpu_baseline(A, x_col, k: int, warmup: int, budget_s: float, dtype):
    """The reference compute_csr (restated in oracle/spmm_oracle.c, bit-pinned against the reference build) on this
    host, same A and the same column-major x the GPU's B was made from: (the oracle's C [m][k], the record)."""
    import numpy as np
    from oracle import oracle as O
    threads, model = cpu_share()
    L = O.lib()
    vals = np.ascontiguousarray(A.values, dtype)
    x = np.ascontiguousarray(x_col, dtype)
    y = np.zeros(A.m * k, dtype)
    fn = L.oracle_spmm_csr_d if dtype == np.float64 else L.oracle_spmm_csr_f

    def call():
        fn(A.row_ptr, A.col_idx, vals, A.m, A.ncols, x, y, k, threads)
    # the reference harness's 100 warm-ups (spmv_bench.cpp:316-320), bounded to ~15 s of CPU time so the default
    # bench finishes in minutes on a box that gives the process few cores
    t0 = time.perf_counter()
    call()
    t_first = time.perf_counter() - t0
    warmup = max(1, min(warmup, int(15.0 / max(t_first, 1e-6))))
    t0 = time.perf_counter()
    for _ in range(warmup - 1):
        call()
    t_warm = time.perf_counter() - t0 + t_first
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 3 or (time.perf_counter() < t_end and len(times) < 100):
        t0 = time.perf_counter()
        call()
        times.append(time.perf_counter() - t0)
    times.sort()
    t = times[len(times) // 2]
    gf = 2.0 * A.nnz * k / t / 1e9
    y_x = y.reshape(A.m, k).copy()             # the oracle's C for this x: the caller checks the GPU's C against it
    # the reference harness's own B (x = 1.0, spmv_bench.cpp:901) as well: BASELINE.md asks for both
    ones = np.ones_like(x)
    fn(A.row_ptr, A.col_idx, vals, A.m, A.ncols, ones, y, k, threads)
    t1 = []
    for _ in range(5):
        t0 = time.perf_counter()
        fn(A.row_ptr, A.col_idx, vals, A.m, A.ncols, ones, y, k, threads)
        t1.append(time.perf_counter() - t0)
    t_ones = sorted(t1)[2]
    return y_x, {"value": round(gf, 3), "unit": "GFLOP/s", "cores": threads, "kind": "port",
            "value_x_ones": round(2.0 * A.nnz * k / t_ones / 1e9, 3),
            "sample": (f"full matrix, same A and x (drand48 seed 42, column-major) as the GPU run; oracle/liboracle.so "
                       f"(C restatement of compute_csr, bit-identical to the reference build); {threads} OpenMP threads "
                       f"(OMP_PROC_BIND=true OMP_PLACES=cores OMP_DYNAMIC=false) on {model}; {warmup} warm-up calls "
                       f"({t_warm:.1f} s) + {len(times)} timed, median {t * 1e3:.1f} ms/call; value_x_ones: the "
                       f"reference harness's x = 1.0, 5 timed calls, median {t_ones * 1e3:.1f} ms/call")}


def cpu_time_once(A, x_col, k: int, dtype, threads: int, budget_s: float):
    """One warm-up + timed calls of the oracle's compute_csr within budget_s (at least one): (median seconds, the
    oracle's C [m][k], which the caller checks the GPU's C against)."""
    import numpy as np
    from oracle import oracle as O
    L = O.lib()
    vals = np.ascontiguousarray(A.values, dtype)
    y = np.zeros(max(A.m, 1) * k, dtype)
    fn = L.oracle_spmm_csr_d if dtype == np.float64 else L.oracle_spmm_csr_f
    fn(A.row_ptr, A.col_idx, vals, A.m, A.ncols, x_col, y, k, threads)
    ts = []
    t_end = time.perf_counter() + budget_s
    while not ts or (time.perf_counter() < t_end and len(ts) < 5):
        t0 = time.perf_counter()
        fn(A.row_ptr, A.col_idx, vals, A.m, A.ncols, x_col, y, k, threads)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], y[: A.m * k].reshape(A.m, k)


def oracle_compare(A, x_col, k: int, got, want, exact, dtype) -> dict:
    """The GPU's C against the oracle's C on the same A and B: rows the engine reports exact (one left-to-right FMA
    chain) must be bit-identical; the rest (split / vector-lane rows) within the normwise contract of SURVEY §8a(ii)
    (|C - C_ref| <= tol * sum_j |a_ij b_jn|, tol 1e-10 fp64 / (len + 1) 2^-24 fp32, doubled: both sides round)."""
    import numpy as np
    iv = np.int64 if got.dtype == np.float64 else np.int32
    same = (np.ascontiguousarray(got).view(iv) == np.ascontiguousarray(want).view(iv)).all(axis=1)
    ex = exact[: A.m].astype(bool)
    out = {"rows_exact": int(ex.sum()), "exact_mismatch": int((ex & ~same).sum()), "rows_inexact": int((~ex).sum()),
           "inexact_outside_tol": 0}
    rows = np.flatnonzero(~ex)
    if len(rows):
        import scipy.sparse as sp
        absB = np.abs(np.asarray(x_col, np.float64).reshape(k, A.ncols).T)      # column-major x -> B [ncols][k]
        absA = sp.csr_matrix((np.abs(A.values.astype(dtype).astype(np.float64)), A.col_idx, A.row_ptr),
                             shape=(A.m, A.ncols))[rows]
        absdot = np.asarray(absA @ absB)
        lens = np.diff(A.row_ptr)[rows].astype(np.float64)
        tol = np.full(len(rows), 1e-10) if dtype == np.float64 else (lens + 1.0) * 2.0 ** -24
        d = np.abs(got[rows].astype(np.float64) - want[rows].astype(np.float64))
        ok_rows = np.all(d <= 2.0 * tol[:, None] * absdot + 1e-300, axis=1)
        out["inexact_outside_tol"] = int((~ok_rows).sum())
    out["ok"] = out["exact_mismatch"] == 0 and out["inexact_outside_tol"] == 0
    return out


def selfcheck(A, B_host_rowmajor, C_dev, k: int, dtype, nsample: int = 256, seed: int = 5) -> dict:
    """numpy recomputation of sampled rows (not the oracle; a sanity check of the run, parity is in tests/).
    B_host_rowmajor: host B [ncols][k], or a callable rows -> B rows (e.g. gathered from HBM)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    m = A.m
    if m == 0:
        return {"rows": 0, "ok": True}
    deg = np.diff(A.row_ptr)
    rows = np.unique(np.concatenate([rng.choice(m, min(nsample, m), replace=False), [int(np.argmax(deg))]]))
    import torch
    got_all = C_dev[torch.from_numpy(rows).to(C_dev.device)].cpu().numpy().astype(np.float64)
    cols = np.unique(np.concatenate([A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]] for r in rows]))
    if callable(B_host_rowmajor):
        bsub = B_host_rowmajor(cols).astype(np.float64)
    else:
        bsub = B_host_rowmajor[cols].astype(np.float64)
    ok = True
    worst = 0.0
    for i, r in enumerate(rows):
        s, e = int(A.row_ptr[r]), int(A.row_ptr[r + 1])
        got = got_all[i]
        bv = bsub[np.searchsorted(cols, A.col_idx[s:e])]
        av = A.values[s:e].astype(dtype).astype(np.float64)
        want = av @ bv if e > s else np.zeros(k)
        absdot = np.abs(av) @ np.abs(bv) if e > s else np.zeros(k)
        tol = 1e-10 if dtype == np.float64 else (e - s + 1) * 2.0 ** -24
        bound = tol * np.maximum(np.abs(want), absdot) + 1e-300
        err = np.abs(got - want) / bound
        worst = max(worst, float(err.max()) if len(err) else 0.0)
        ok = ok and bool(np.all(np.isfinite(got))) and bool(np.all(err <= 1.0 + 1e-9))
    return {"rows": int(len(rows)), "ok": ok, "max_err_over_bound": round(worst, 6)}


def load_pmc_dataset(path: str, k: int, dtype: str) -> dict:
    """gen line -> per-launch PMC record of THIS engine build, from profiles/pmc_dataset_latest.json ({"records":
    [...]}, written by tools/pmc_dataset.py publish); {} when none match (the record then carries traffic null)."""
    p = Path(path)
    if not p.exists():
        return {}
    try:
        recs = json.loads(p.read_text()).get("records", [])
    except ValueError:
        return {}
    sha = engine_sha256()
    return {r["gen"]: r for r in recs
            if r.get("engine_sha256") == sha and r.get("k") == k and r.get("dtype") == dtype}


def pctl(v: list, q: float) -> float:
    s = sorted(v)
    return s[min(len(s) - 1, int(q * len(s)))] if s else float("nan")


def run_lines(lines, K: int, dtype: str, iters: int, warmup: int, torch, S, np, cpu_budget_s: float = 0.0,
              cpu_each_s: float = 0.0, pmc: dict | None = None, names: dict | None = None, log=True) -> dict:
    """Time every generator line at K (HBM-resident A, B, C; HIP events on the launch stream), self-check sampled
    rows, attach PMC traffic / the gather ceiling when `pmc` has the line; the CPU baseline runs on the matrices in
    sample order while `cpu_budget_s` lasts (and `cpu_each_s` per matrix when set: twins).  Matrix generation runs
    one line ahead on a host thread (the generator releases the GIL), so the GPU does not wait for it."""
    from concurrent.futures import ThreadPoolExecutor
    dev_index = torch.cuda.current_device()          # this rank's GPU (set by main before any record runs)
    dev = torch.device("cuda", dev_index)
    tdt = torch.float64 if dtype == "f64" else torch.float32
    npdt = np.float64 if dtype == "f64" else np.float32
    dt_code = S.F64 if dtype == "f64" else S.F32
    stream = torch.cuda.current_stream(dev)
    threads, model = cpu_share()
    pmc = pmc or {}
    recs, bad = [], 0
    cpu_left = cpu_budget_s
    t_start = time.perf_counter()
    ex = ThreadPoolExecutor(max_workers=1)
    fut = ex.submit(lambda l: S.generate(S.gen_params(l)), lines[0]) if lines else None
    for i, line in enumerate(lines):
        A = fut.result()
        fut = ex.submit(lambda l: S.generate(S.gen_params(l)), lines[i + 1]) if i + 1 < len(lines) else None
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdt), A.m, A.ncols, A.nnz, K, dev_index)
        g = torch.Generator(device=dev)
        g.manual_seed(42)
        B = torch.rand((max(A.ncols, 1), K), generator=g, device=dev, dtype=tdt)
        C = torch.empty((max(A.m, 1), K), device=dev, dtype=tdt)
        def launch():
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), K, stream.cuda_stream)
        for _ in range(warmup):
            launch()
        torch.cuda.synchronize()
        t = timed_launches(torch, stream, launch, iters) * 1e-3
        chk = selfcheck(A, lambda cols: B[torch.from_numpy(cols).to(dev)].cpu().numpy(), C, K, npdt, nsample=32)
        bad += 0 if chk["ok"] else 1
        b = S.bytes_alg(A.m, A.ncols, A.nnz, K, dt_code)
        rec = {"gen": line, "m": int(A.m), "nnz": int(A.nnz), "ms": t * 1e3, "flops": 2.0 * A.nnz * K,
               "bytes_alg": b, "frac": b / t / 1e9 / HBM_PEAK_GBS, "gflops": 2.0 * A.nnz * K / t / 1e9,
               "tiles": int(mf.info()[19]), "tile_mode": mf.tile_info()["mode"], "selfcheck_ok": chk["ok"]}
        if names:
            rec["name"] = names.get(line)
        pm = pmc.get(line)
        if pm and pm.get("nnz") == A.nnz:
            rec["traffic"] = pm["traffic_bytes"]
            ach = achievable(t * 1e3, pm["traffic_bytes"], pm.get("tcc_req"), float(A.ncols) * K * (8 if dtype == "f64" else 4),
                             b)
            rec["frac_of_achievable"] = ach["frac_of_achievable"] if ach else None
        if (cpu_left > 0 or cpu_each_s > 0) and A.nnz > 0:
            t0 = time.perf_counter()
            x_col = np.ascontiguousarray(B.t().cpu().numpy()).ravel()[: A.ncols * K]
            tc, want = cpu_time_once(A, x_col, K, npdt, threads, cpu_each_s if cpu_each_s > 0 else min(cpu_left, 2.0))
            rec["cpu_ms"] = tc * 1e3
            # the CPU baseline's own output checks this run's C: bit-exact on the rows the engine reports exact
            rec["oracle_check"] = oracle_compare(A, x_col, K, C[: A.m].cpu().numpy(), want, mf.exact_rows(), npdt)
            bad += 0 if rec["oracle_check"]["ok"] else 1
            cpu_left -= time.perf_counter() - t0
            del x_col
        recs.append(rec)
        mf.close()
        del B, C, A
        if log:
            print(f"[{i + 1}/{len(lines)}] {line}: {rec['gflops']:.1f} GFLOP/s frac {rec['frac']:.3f}"
                  + (f" cpu {rec['cpu_ms']:.1f} ms" if "cpu_ms" in rec else ""), file=sys.stderr, flush=True)
    ex.shutdown()
    return {"recs": recs, "bad": bad, "wall_s": time.perf_counter() - t_start, "threads": threads, "model": model}


def summarize(res: dict, K: int) -> dict:
    recs = res["recs"]
    tot_f = sum(r["flops"] for r in recs)
    tot_s = sum(r["ms"] for r in recs) * 1e-3
    tot_b = sum(r["bytes_alg"] for r in recs)
    fr = [r["frac"] for r in recs]
    out = {"matrices": len(recs), "value": round(tot_f / tot_s / 1e9, 3), "unit": "GFLOP/s",
           "median_gflops": round(pctl([r["gflops"] for r in recs], 0.5), 2),
           "roofline": {"bound": "hbm", "achieved": round(tot_b / tot_s / 1e9, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(tot_b / tot_s / 1e9 / HBM_PEAK_GBS, 4),
                        "median_frac": round(pctl(fr, 0.5), 4), "p10_frac": round(pctl(fr, 0.1), 4),
                        "p90_frac": round(pctl(fr, 0.9), 4)},
           "mean_ms_per_matrix": round(tot_s * 1e3 / max(len(recs), 1), 5),
           "selfcheck_failures": res["bad"], "wall_s": round(res["wall_s"], 1)}
    with_t = [r for r in recs if "traffic" in r]
    if with_t:
        tt = sum(r["traffic"] for r in with_t)
        ts = sum(r["ms"] for r in with_t) * 1e-3
        fa = [r["frac_of_achievable"] for r in with_t if r.get("frac_of_achievable")]
        out["roofline"]["traffic"] = tt / len(with_t)
        out["roofline"]["traffic_note"] = (f"mean PMC past-L2 bytes per launch over the {len(with_t)} matrices with "
                                           "records for this engine build (profiles/pmc_dataset_latest.json)")
        out["roofline"]["traffic_gbs_aggregate"] = round(tt / ts / 1e9, 1)
        out["roofline"]["achievable"] = {"median_frac_of_achievable": round(pctl(fa, 0.5), 4) if fa else None,
                                         "p10": round(pctl(fa, 0.1), 4) if fa else None,
                                         "p90": round(pctl(fa, 0.9), 4) if fa else None, "matrices": len(fa)}
    else:
        out["roofline"]["traffic"] = None
        out["roofline"]["achievable"] = None
    cp = [r for r in recs if "cpu_ms" in r]
    if cp:
        cf = sum(r["flops"] for r in cp)
        cs = sum(r["cpu_ms"] for r in cp) * 1e-3
        gs = sum(r["ms"] for r in cp) * 1e-3
        out["cpu_baseline"] = {
            "value": round(cf / cs / 1e9, 3), "unit": "GFLOP/s", "cores": res["threads"], "kind": "port",
            "sample": (f"{len(cp)} of the {len(recs)} matrices (in sample order, time-bounded), same A and B as the GPU "
                       f"run; oracle/liboracle.so (C restatement of compute_csr, bit-identical to the reference build), "
                       f"{res['threads']} OpenMP threads on {res['model']}; 1 warm-up + median of timed calls each; "
                       f"aggregate = sum flops / sum time; GPU aggregate on the same subset "
                       f"{cf / gs / 1e9:.1f} GFLOP/s")}
    else:
        out["cpu_baseline"] = None
    oc = [r["oracle_check"] for r in recs if "oracle_check" in r]
    out["oracle_check"] = {
        "matrices": len(oc), "rows_exact": sum(c["rows_exact"] for c in oc),
        "exact_rows_not_bitexact": sum(c["exact_mismatch"] for c in oc),
        "rows_inexact": sum(c["rows_inexact"] for c in oc),
        "inexact_rows_outside_tol": sum(c["inexact_outside_tol"] for c in oc),
        "note": ("every row of the CPU-baselined matrices against the oracle's C on the same A and B: bit-identical "
                 "where the engine reports the row exact, else within 2x the normwise tolerance")} if oc else None
    return out


def run_dataset_record(args, torch, S, np, iters: int | None = None, warmup: int | None = None, offset: int | None = None,
                       cpu: bool = True, pmc_on: bool = True) -> dict:
    """The metric's own workload: every stride-th medium-dataset line from `offset`, `iters` timed launches each."""
    from spmm_amd.datasets import medium_dataset_lines
    iters = args.dataset_iters if iters is None else iters
    warmup = args.dataset_warmup if warmup is None else warmup
    offset = args.dataset_offset if offset is None else offset
    lines = medium_dataset_lines()[offset::args.dataset_stride]
    pmc = load_pmc_dataset(args.pmc_dataset, args.k, args.dtype) if pmc_on else {}
    res = run_lines(lines, args.k, args.dtype, iters, warmup, torch, S, np,
                    cpu_budget_s=0.0 if (args.no_cpu_baseline or not cpu) else args.dataset_cpu_seconds, pmc=pmc)
    rec = summarize(res, args.k)
    if args.dataset_out:
        rank = int(os.environ.get("RANK", "0"))
        path = args.dataset_out + (f".r{rank}" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else "")
        with open(path, "w") as f:
            for r in res["recs"]:
                f.write(json.dumps(r) + "\n")
    rec.update({"metric": METRIC, "scaling": "single-gpu", "dtype": args.dtype,
                "workload": f"every {args.dataset_stride}th line of synthetic_matrices_medium_dataset from "
                            f"{offset} ({len(lines)} matrices), K={args.k}",
                "iters_per_matrix": iters, "warmup_per_matrix": warmup,
                "ms_per_pass": round(sum(r["ms"] for r in res["recs"]), 5),
                "flops_per_pass": sum(r["flops"] for r in res["recs"]),
                "bytes_alg_per_pass": sum(r["bytes_alg"] for r in res["recs"]),
                "nnz_total": int(sum(r["nnz"] for r in res["recs"]))})
    return rec


def run_medium_sample(args, torch, S, np):
    """config 3 at N=1: a strided sample of the medium dataset as the line itself."""
    torch.cuda.set_device(0)
    d = run_dataset_record(args, torch, S, np)
    line = {"metric": METRIC, "value": d["value"], "unit": "GFLOP/s", "n_gpus": 1, "steps": args.dataset_iters,
            "warmup": args.dataset_warmup, "ms_per_step": d["mean_ms_per_matrix"],
            "higher_is_better": True, "scaling": "single-gpu", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (own generator, seeded; A values U[0.5,1.5), B torch.rand(seed 42))",
            "config": {"workload": "medium-sample: " + d["workload"], "k": args.k, "parallelism": "single-gpu"},
            "roofline": d["roofline"], "cpu_baseline": d["cpu_baseline"], "oracle_check": d.get("oracle_check"),
            "setup": {"wall_s": d["wall_s"], "selfcheck_failures": d["selfcheck_failures"]}}
    print(json.dumps(line), flush=True)
    return 0 if d["selfcheck_failures"] == 0 else 1


def run_twins(args, torch, S, np):
    """config 5: the 52 validation twins (reference config.sh:283-339) at K, fp64 and fp32, one GPU; a CPU baseline
    on every twin in the same run (oracle compute_csr, time-bounded per twin)."""
    from spmm_amd.datasets import twins
    torch.cuda.set_device(0)
    tw = twins()
    names = {line: name for name, line in tw.items()}
    lines = list(tw.values())
    per = {}
    bad = 0
    for dt in ("f64", "f32"):
        res = run_lines(lines, args.k, dt, args.dataset_iters, args.dataset_warmup, torch, S, np,
                        cpu_each_s=0.0 if args.no_cpu_baseline else args.twins_cpu_seconds, names=names)
        s = summarize(res, args.k)
        s["per_twin"] = [{"name": r["name"], "nnz": r["nnz"], "ms": round(r["ms"], 5), "gflops": round(r["gflops"], 1),
                          "frac": round(r["frac"], 4), "cpu_gflops": round(r["flops"] / r["cpu_ms"] / 1e6, 2)
                          if r.get("cpu_ms") else None, "tiles": r["tiles"], "tile_mode": r["tile_mode"],
                          "oracle_ok": r["oracle_check"]["ok"] if "oracle_check" in r else None}
                         for r in res["recs"]]
        bad += res["bad"]
        per[dt] = s
    line = {"metric": "GFLOP/s, validation twins (config 5), CSR SpMM K=32, aggregate over the twins",
            "value": per["f64"]["value"], "unit": "GFLOP/s", "n_gpus": 1, "steps": args.dataset_iters,
            "warmup": args.dataset_warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "single-gpu",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic twins (own generator on the reference's twin lines; A U[0.5,1.5), B torch.rand(42))",
            "config": {"workload": f"twins: {len(lines)} validation twins (spmm_amd/validation_twins.json), K={args.k}",
                       "k": args.k, "parallelism": "single-gpu"},
            "roofline": per["f64"]["roofline"], "cpu_baseline": per["f64"]["cpu_baseline"], "per_dtype": per,
            "setup": {"selfcheck_failures": bad}}
    print(json.dumps(line), flush=True)
    return 0 if bad == 0 else 1


def run_pipeline(args, torch, S, np):
    """one reference compute() step on the engine, graph-captured, fp32 by default."""
    from spmm_amd import pipeline as P
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    npdt = np.float64 if args.dtype == "f64" else np.float32
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    m, k, n = args.pipe_m, args.pipe_k, args.pipe_n
    w = [P.dlmc_like_weight(m, k, args.pipe_density, 100 + i) for i in range(3)]
    mask = P.band_and_random_mask(m, args.pipe_mask_density, args.pipe_band, 107)
    x = S.drand48(42, k * n).reshape(k, n)
    pipe = P.SparseAttentionPipeline(*w, mask, n, npdt, args.pipe_mode)
    bx = torch.from_numpy(x.astype(npdt)).to(dev)
    bufs = [torch.zeros((m, n), dtype=tdt, device=dev) for _ in range(3)]
    y = torch.zeros(mask.nnz, dtype=tdt, device=dev)
    out = torch.zeros((m, n), dtype=tdt, device=dev)
    s = torch.cuda.Stream(dev)
    ptrs = (bx.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr(), y.data_ptr(), out.data_ptr())
    with torch.cuda.stream(s):
        for _ in range(3):
            pipe.run_device(*ptrs, s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pipe.run_device(*ptrs, s.cuda_stream)
    for _ in range(args.warmup):
        g.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(s)
    with torch.cuda.stream(s):
        for _ in range(args.steps):
            g.replay()
    ev1.record(s)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    # parity of this run, stage by stage against the oracle on the GPU's own stage inputs (test infrastructure
    # as the checker): SDDMM bit-exact; K/Q/V on the rows the engine reports exact
    ok = True
    for t, a, b in zip("KQV", w, bufs):
        ex = pipe.mf[t].exact_rows()
        want = O.spmm_rowmajor(a.row_ptr, a.col_idx, a.values.astype(npdt), k, x.astype(npdt))
        ok = ok and np.array_equal(b.cpu().numpy()[ex], want[ex])
    if not args.pipe_mode & 2:
        yo = O.sddmm(mask.row_ptr, mask.col_idx, mask.values.astype(npdt), bufs[1].cpu().numpy(),
                     bufs[0].cpu().numpy(), args.pipe_mode & 1)
        ok = ok and np.array_equal(y.cpu().numpy(), yo)
    flops = pipe.flops
    # CPU baseline: the oracle's stages (the reference compute() step's arithmetic) on this host, bounded sample
    cpu = None
    if not args.no_cpu_baseline:
        threads, model = cpu_share()
        ts = []
        t_end = time.perf_counter() + args.cpu_seconds
        while len(ts) < 3 or (time.perf_counter() < t_end and len(ts) < 50):
            t1 = time.perf_counter()
            Kc, Qc, Vc = (O.spmm_rowmajor(a.row_ptr, a.col_idx, a.values.astype(npdt), k, x.astype(npdt)) for a in w)
            yc = O.sddmm(mask.row_ptr, mask.col_idx, mask.values.astype(npdt), Qc, Kc, args.pipe_mode & 1)
            O.spmm_rowmajor(mask.row_ptr, mask.col_idx, yc, m, Vc)
            ts.append(time.perf_counter() - t1)
        ts.sort()
        cpu = {"value": round(flops / ts[len(ts) // 2] / 1e9, 3), "unit": "GFLOP/s", "cores": threads, "kind": "port",
               "sample": f"one pipeline step per call, oracle C restatement (SpMMs {threads} OpenMP threads, SDDMM "
                         f"serial) on {model}; {len(ts)} calls, median {ts[len(ts) // 2] * 1e3:.2f} ms"}
    line = {
        "metric": "GFLOP/s, sparse-attention pipeline step (SpMM K,Q,V + SDDMM + SpMM), reference formula",
        "value": round(flops / (step_ms * 1e-3) / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 5), "higher_is_better": True, "scaling": "single-gpu",
        "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (DLMC-like random-pruned weights U[-1,1), seeded band+random mask, x drand48(42))",
        "config": {"workload": f"pipeline: m={m} k={k} n={n} weight density {args.pipe_density} mask density "
                               f"{args.pipe_mask_density} band {args.pipe_band} sddmm flags {args.pipe_mode}",
                   "nnz": [a.nnz for a in w] + [mask.nnz], "parallelism": "single-gpu"},
        "wall_ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "cpu_baseline": cpu, "setup": {"stages_bitexact_vs_oracle": ok},
    }
    print(json.dumps(line), flush=True)
    pipe.close()
    return 0 if ok else 1


def run_multi_handle(args, torch, S, np, p, K: int, npdtype, B, Bh, devices: list, stream) -> dict:
    """The C-ABI multi-GPU handle in ONE process (spmm_hip_create_multi, include/spmm_hip.h) -- the path the
    reference-harness plugin takes with SPMM_HIP_NGPUS (integration/spmm_kernel_hip.cpp) -- over the same global
    matrix and the same reference-partitioner shards as the torch.distributed ranks.  B (on device 0) is replicated
    once by each broadcast the handle offers, side by side (SURVEY §8e "benchmark both"): root -> peer
    hipMemcpyPeerAsync over xGMI, and one grouped RCCL broadcast (SPMM_HIP_BCAST=rccl, distinct devices only); then
    spmm_hip_run_sharded is timed with HIP events on the caller's stream (every shard's stream forks from it and joins
    back into it), C left sharded like the distributed loop.  Afterwards C is gathered to device 0 once
    (spmm_hip_run_device) and self-checked.  Rank 0 only, after the distributed measurement."""
    A = S.generate(p)
    flops = 2.0 * A.nnz * K
    bbytes = float(A.ncols) * K * np.dtype(npdtype).itemsize
    ndist = len(set(devices))
    sp = stream.cuda_stream
    out = {"devices": devices, "nnz": int(A.nnz), "b_bytes": bbytes, "modes": {}}

    def sync_all():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)
    for mode in ("peer", "rccl"):
        if mode == "rccl" and ndist != len(devices):
            out["modes"][mode] = {"skipped": "RCCL broadcast needs distinct devices (shards share a GPU in this run)"}
            continue
        old = os.environ.get("SPMM_HIP_BCAST")
        os.environ.pop("SPMM_HIP_BCAST", None)
        if mode == "rccl":
            os.environ["SPMM_HIP_BCAST"] = "rccl"
        try:
            mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdtype), A.m, A.ncols, A.nnz, K,
                                 devices=devices)
        except S.SpmmHipError as e:
            out["modes"][mode] = {"skipped": str(e)}
            continue
        finally:
            os.environ.pop("SPMM_HIP_BCAST", None)
            if old is not None:
                os.environ["SPMM_HIP_BCAST"] = old
        mf.broadcast_b(B.data_ptr(), S.B_ROW_MAJOR, K, sp)
        sync_all()
        tb = []
        for _ in range(5):
            t0 = time.perf_counter()
            mf.broadcast_b(B.data_ptr(), S.B_ROW_MAJOR, K, sp)
            sync_all()
            tb.append(time.perf_counter() - t0)
        t_b = sorted(tb)[2]
        for _ in range(args.warmup):
            mf.run_sharded(K, sp)
        sync_all()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            mf.run_sharded(K, sp)
        e1.record(stream)
        sync_all()
        ms = e0.elapsed_time(e1) / max(args.steps, 1)
        Cf = torch.empty((max(A.m, 1), K), device=B.device, dtype=B.dtype)
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cf.data_ptr(), K, sp)
        sync_all()
        chk = selfcheck(A, Bh, Cf, K, npdtype)
        out["modes"][mode] = {"bcast_B_s": round(t_b, 5),
                              "bcast_GBs": round(bbytes * (ndist - 1) / t_b / 1e9, 1) if ndist > 1 else None,
                              "ms_per_step": round(ms, 5), "value": round(flops / (ms * 1e-3) / 1e9, 3),
                              "unit": "GFLOP/s", "shards": mf.ngpus()[0], "selfcheck_ok": bool(chk["ok"])}
        mf.close()
        del Cf
    return out


def dump_c(path: str, C_all, exact_all, k: int) -> None:
    """Row sample of C (every 101st row and the last row) + the exact mask of those rows (tests compare runs)."""
    import numpy as np
    import torch
    m = C_all.shape[0]
    rows = np.unique(np.concatenate([np.arange(0, m, 101), [m - 1]])).astype(np.int64)
    c = C_all[torch.from_numpy(rows).to(C_all.device)].cpu().numpy()
    np.savez(path, rows=rows, c=c, exact=np.asarray(exact_all)[rows], k=np.int64(k))


class Ctx:
    """Per-process run context: world, rank, process group, device, and the imported modules."""

    def __init__(self, args, N, rank, dist, dev, dev_index, torch, S, np, sharding):
        self.args, self.N, self.rank, self.dist = args, N, rank, dist
        self.dev, self.dev_index, self.torch, self.S, self.np, self.sharding = dev, dev_index, torch, S, np, sharding

    def barrier(self):
        self.torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()
        self.torch.cuda.synchronize()


def measure_line(ctx: Ctx, gen: str, scaling: str, workload: str, cpu: bool, e2e: bool, multi: bool,
                 dump: str | None) -> tuple[dict, bool]:
    """One generator line as one SpMM per step: the global matrix (scaling "weak": the line's shape N times over;
    "strong": the line itself) split into N nnz-balanced row ranges with the reference partitioner, this rank's rows
    generated and planned, B drand48(42) broadcast once, --warmup untimed and --steps timed launches bracketed by a
    barrier + synchronize on both sides, value from the max over ranks of the HIP-event time.  Returns (record, ok)
    on every rank (the record is complete on rank 0)."""
    args, N, rank, dist, dev, torch, S, np = ctx.args, ctx.N, ctx.rank, ctx.dist, ctx.dev, ctx.torch, ctx.S, ctx.np
    sharding = ctx.sharding
    K = args.k
    tdtype = torch.float64 if args.dtype == "f64" else torch.float32
    npdtype = np.float64 if args.dtype == "f64" else np.float32

    # ---- this rank's shard of the global matrix (nnz-balanced row split, a8 partitioner)
    t0 = time.perf_counter()
    p = sharding.weak_scaled_params(gen, N) if (N > 1 and scaling == "weak") else S.gen_params(gen)
    rp_global = S.generate_row_ptr(p)
    nnz_total = int(rp_global[-1])
    bounds = [S.partition_rows(rp_global, nnz_total, N, w) for w in range(N)]
    r0, r1 = bounds[rank]
    A = S.generate_rows(p, r0, r1) if N > 1 else S.generate(p)
    per_rank = [int(rp_global[e] - rp_global[s]) for s, e in bounds]
    imbalance = max(per_rank) / (sum(per_rank) / N) if nnz_total else 1.0
    del rp_global
    t_gen = time.perf_counter() - t0
    ncols = int(p.nr_cols)

    t0 = time.perf_counter()
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdtype), A.m, ncols, A.nnz, K, ctx.dev_index)
    t_plan = time.perf_counter() - t0

    # ---- B: drand48(42) column-major x on rank 0 (the reference harness convention), row-major in HBM, broadcast
    x_col = Bh = None
    if rank == 0:
        x_col = S.drand48(42, ncols * K)
        Bh = np.ascontiguousarray(x_col.reshape(K, ncols).T).astype(npdtype)
        B = torch.from_numpy(Bh).to(dev)
    else:
        B = torch.empty((ncols, K), device=dev, dtype=tdtype)
    t_bcast = 0.0
    if dist is not None:
        ctx.barrier()
        tb = time.perf_counter()
        sharding.broadcast_b(dist, B)        # RCCL over xGMI, once at setup
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - tb
    C = torch.empty((max(A.m, 1), K), device=dev, dtype=tdtype)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def step():
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), K, sptr)

    for _ in range(args.warmup):
        step()
    ctx.barrier()
    t0 = time.perf_counter()
    kern_ms = timed_launches(torch, stream, step, args.steps)      # HIP events on the launch stream, per step
    ctx.barrier()
    elapsed = time.perf_counter() - t0                             # barrier-inclusive wall time of the K steps
    bytes_launch = S.bytes_alg(A.m, ncols, A.nnz, K, S.F64 if args.dtype == "f64" else S.F32)
    kern_all, bytes_all = [kern_ms], [bytes_launch]
    if dist is not None:
        kt = sharding.gather_scalars(dist, [kern_ms, bytes_launch, elapsed], dev)
        kern_all = [v[0] for v in kt]
        bytes_all = [v[1] for v in kt]
        elapsed = max(v[2] for v in kt)
    slow = int(np.argmax(kern_all))
    kern_max_ms = kern_all[slow]

    # ---- C all-gather, once, timed (validation / hand-back path, never inside the timed loop)
    t_gather = None
    exact = mf.exact_rows()
    c_all, exact_all = C[: A.m], exact
    if dist is not None:
        counts = [e - s for s, e in bounds]
        ctx.barrier()
        tg = time.perf_counter()
        c_all = sharding.allgather_rows(dist, C[: max(A.m, 1)], counts)
        torch.cuda.synchronize()
        t_gather = time.perf_counter() - tg
        ex_t = torch.from_numpy(exact.astype(np.uint8).reshape(-1, 1)).to(dev)
        exact_all = sharding.allgather_rows(dist, ex_t if A.m else torch.zeros((1, 1), dtype=torch.uint8, device=dev),
                                            counts).cpu().numpy().ravel().astype(bool)
    if rank == 0 and dump:
        dump_c(dump, c_all, exact_all, K)
    del c_all

    # ---- self-check on every rank (B rows for the check: rank 0 has them on the host; others copy from HBM)
    Bh_chk = Bh if rank == 0 else B.cpu().numpy()
    chk = selfcheck(A, Bh_chk, C, K, npdtype)
    ok_all = chk["ok"]
    if dist is not None:
        ok_all = all(v[0] == 0 for v in sharding.gather_scalars(dist, [0.0 if chk["ok"] else 1.0], dev))

    flops_step = 2.0 * nnz_total * K
    gflops = flops_step / (kern_max_ms * 1e-3) / 1e9
    # the slowest rank bounds the step: its bytes over its time (one definition at every N: the rank's rows and
    # nonzeros with the global column count)
    achieved = bytes_all[slow] / (kern_max_ms * 1e-3) / 1e9
    traffic = l2_req = None
    try:
        pm = json.loads(Path(args.pmc_json).read_text())
        if (pm.get("workload") == gen and pm.get("k") == K and pm.get("dtype") == args.dtype and N == 1
                and pm.get("nnz") == A.nnz and pm.get("engine_sha256") == engine_sha256()):
            traffic = pm.get("hbm_bytes_per_launch")
            cc = pm.get("counters_per_launch", {})
            if "TCC_HIT_sum" in cc and "TCC_MISS_sum" in cc:
                l2_req = cc["TCC_HIT_sum"] + cc["TCC_MISS_sum"]
    except Exception:
        pass
    ach = achievable(kern_max_ms, traffic, l2_req, float(ncols) * K * (8 if args.dtype == "f64" else 4),
                     bytes_all[slow])

    # ---- plugin end to end (N=1): host x / y through the reference contract (H2D + transpose + kernel + D2H)
    e2e_rec = None
    if N == 1 and e2e:
        y = np.empty(A.m * K, npdtype)
        xh = x_col.astype(npdtype)
        mf.spmm(xh, y, K)
        te = []
        for _ in range(3):
            t1 = time.perf_counter()
            mf.spmm(xh, y, K)
            te.append(time.perf_counter() - t1)
        lt = mf.last_times()
        e2e_rec = {"ms_per_call": round(sorted(te)[1] * 1e3, 3),
                   "gflops": round(flops_step / sorted(te)[1] / 1e9, 2),
                   "events_ms": {k_: round(v, 4) for k_, v in lt.items()},
                   "note": "pageable host buffers; PCIe-inclusive, never the headline value"}
        del y, xh

    cpu_rec = None
    if rank == 0 and N == 1 and cpu and not args.no_cpu_baseline:
        want = None
        try:
            want, cpu_rec = cpu_baseline(A, x_col, K, args.cpu_warmup, args.cpu_seconds, npdtype)
        except Exception as e:  # the baseline is reported, never required
            cpu_rec = {"value": None, "unit": "GFLOP/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}
        if want is not None:
            # the baseline's own C checks this run's C over every row (bit-exact where the engine reports exact); a
            # failure of the check itself fails the record, it is never reported as a baseline failure
            try:
                cpu_rec["oracle_check"] = oracle_compare(A, x_col, K, C[: A.m].cpu().numpy(), want, exact, npdtype)
            except Exception as e:
                cpu_rec["oracle_check"] = {"ok": False, "error": f"{type(e).__name__}: {e}"}
            ok_all = ok_all and cpu_rec["oracle_check"]["ok"]
            del want
    mf.close()
    del C

    # ---- N>1: the in-process multi-GPU handle of the C ABI over the same matrix (rank 0; the others wait)
    multi_rec = None
    if dist is not None and multi and not args.no_multi_handle:
        if rank == 0:
            devs = [0] * N if args.dist_backend == "gloo" else list(range(N))
            try:
                multi_rec = run_multi_handle(args, torch, S, np, p, K, npdtype, B, Bh, devs, stream)
            except Exception as e:   # reported, the distributed record stands on its own
                multi_rec = {"error": f"{type(e).__name__}: {e}"}
        dist.barrier()
    del B

    rec = {
        "metric": METRIC,
        "value": round(gflops, 3),
        "unit": "GFLOP/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(kern_max_ms, 5),
        "higher_is_better": True,
        "scaling": scaling if N > 1 else "single-gpu",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (own generator, seeded; A values U[0.5,1.5), B drand48(42))",
        "config": {"workload": f"{workload}: csr_spmm gen='{gen}'"
                               + (f" x{N} stacked (weak)" if scaling == "weak" and N > 1 else "")
                               + f", K={K}",
                   "nnz_total": nnz_total, "rows_total": int(p.nr_rows), "cols": ncols, "k": K,
                   "nnz_per_rank": per_rank, "imbalance_max_over_mean": round(imbalance, 4),
                   "parallelism": f"row-shard{N}" if N > 1 else "single-gpu",
                   "dist_backend": args.dist_backend if N > 1 else None},
        "timing": "value = 2*nnz*K / (max over ranks of the HIP-event time per step of the K timed steps, launch "
                  "stream); wall_ms_per_step = barrier-inclusive host wall time, max over ranks",
        "wall_ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 5),
        "hbm_gbs_alg": round(achieved, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_gbs": None if traffic is None else round(traffic / (kern_max_ms * 1e-3) / 1e9, 1),
                     "achievable": ach,
                     "bytes_alg_per_launch": bytes_all[slow], "kernel_ms_per_launch": round(kern_max_ms, 5),
                     "kernel_ms_per_rank": [round(v, 5) for v in kern_all], "slowest_rank": slow},
        "cpu_baseline": cpu_rec,
        "plugin_e2e": e2e_rec,
        "multi_handle": multi_rec,
        "setup": {"gen_s": round(t_gen, 2), "plan_s": round(t_plan, 2), "bcast_B_s": round(t_bcast, 4),
                  "bcast_B_s_modes": None if multi_rec is None or "modes" not in multi_rec else
                  {"torch.distributed rccl (one process per GPU)": round(t_bcast, 4),
                   **{f"multi-handle {m_}": v_.get("bcast_B_s") for m_, v_ in multi_rec["modes"].items()}},
                  "allgather_C_s": None if t_gather is None else round(t_gather, 4),
                  "selfcheck": chk, "selfcheck_all_ranks_ok": ok_all},
    }
    return rec, ok_all


def run_dataset_line(ctx: Ctx) -> tuple[dict, bool]:
    """The default line: the medium-dataset sample as the value (every rank its own stride sample at N > 1), with
    the config-2 record (N = 1) or the config-4 strong split and the config-2 weak record (N > 1) beside it."""
    args, N, rank, torch, S, np = ctx.args, ctx.N, ctx.rank, ctx.torch, ctx.S, ctx.np
    from spmm_amd.datasets import CONFIG2_LINE, CONFIG4_LINE
    ok = True
    sub = {}
    # ---- sub-records first (they allocate and free whole-GPU buffers; the dataset pass then runs on a clean heap)
    if N == 1 and not args.no_config2:
        rec, ok2 = measure_line(ctx, CONFIG2_LINE, "strong", "config2", cpu=True, e2e=True, multi=False,
                                dump=args.dump_c)
        sub["config2"] = rec
        ok = ok and ok2
    if N > 1 and not args.no_config4:
        rec, ok4 = measure_line(ctx, args.strong_gen or CONFIG4_LINE, "strong", "config4", cpu=False, e2e=False,
                                multi=False, dump=args.dump_c_strong)
        sub["config4_strong"] = rec
        ok = ok and ok4
    if N > 1 and not args.no_config2:
        rec, ok2 = measure_line(ctx, CONFIG2_LINE, "weak", "config2", cpu=False, e2e=False, multi=True,
                                dump=args.dump_c)
        sub["config2_weak"] = rec
        ok = ok and ok2

    # ---- the dataset pass (one step = every matrix of the rank's sample once)
    ds = None
    if not args.no_dataset:
        offset = args.dataset_offset + (rank * args.dataset_stride) // N
        ctx.barrier()
        t0 = time.perf_counter()
        ds = run_dataset_record(args, torch, S, np, iters=args.steps, warmup=args.warmup, offset=offset,
                                cpu=(rank == 0 and N == 1), pmc_on=(N == 1))
        wall = time.perf_counter() - t0
        ctx.barrier()
        mine = [ds["ms_per_pass"], ds["flops_per_pass"], ds["bytes_alg_per_pass"], float(ds["matrices"]),
                float(ds["selfcheck_failures"]), wall]
        allr = ctx.sharding.gather_scalars(ctx.dist, mine, ctx.dev) if ctx.dist is not None else [mine]
        ds["selfcheck_failures_all_ranks"] = int(sum(v[4] for v in allr))
        ok = ok and ds["selfcheck_failures_all_ranks"] == 0
        ms = [v[0] for v in allr]
        slow = int(np.argmax(ms))
        flops = sum(v[1] for v in allr)
        ds["ranks"] = [{"ms_per_pass": round(v[0], 5), "gflops": round(v[1] / (v[0] * 1e-3) / 1e9, 3),
                        "matrices": int(v[3]), "wall_s": round(v[5], 1)} for v in allr]
        ds["value_all_ranks"] = round(flops / (ms[slow] * 1e-3) / 1e9, 3)
        ds["ms_per_step_max_over_ranks"] = round(ms[slow], 5)
        ds["slowest_rank"] = slow
    if rank != 0:
        return {}, ok

    if ds is None:   # sub-records only (tests, PMC tools): the first one is the line
        key = next(iter(sub))
        line = dict(sub.pop(key))
        line["sub_records"] = sub
        return line, ok
    data_desc = "synthetic (own generator, seeded; A values U[0.5,1.5), B torch.rand(seed 42) per matrix)"
    n_mat = sum(r["matrices"] for r in ds["ranks"])
    line = {
        "metric": METRIC,
        "value": ds["value_all_ranks"],
        "unit": "GFLOP/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ds["ms_per_step_max_over_ranks"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": data_desc,
        "config": {"workload": (f"synthetic_matrices_medium_dataset, every {args.dataset_stride}th line"
                                + (f" from {args.dataset_offset}" if N == 1 else
                                   f", rank r from offset {args.dataset_offset} + r*{args.dataset_stride}/{N}")
                                + f" ({n_mat} matrices), CSR SpMM K={args.k} {args.dtype}"),
                   "matrices": n_mat, "matrices_per_rank": [r["matrices"] for r in ds["ranks"]],
                   "k": args.k, "parallelism": f"matrix-shard{N}" if N > 1 else "single-gpu",
                   "dist_backend": args.dist_backend if N > 1 else None},
        "timing": ("one step = one SpMM over every matrix of the rank's sample; per matrix --warmup untimed and "
                   "--steps HIP-event-timed launches on the launch stream (behind a GPU pre-roll); ms_per_step = sum "
                   "over matrices of the per-launch time, max over ranks; value = flops of all ranks / ms_per_step"),
        "roofline": ds["roofline"],
        "cpu_baseline": ds["cpu_baseline"],
        "oracle_check": ds.get("oracle_check"),
        "dataset": {k_: v_ for k_, v_ in ds.items() if k_ not in ("roofline", "cpu_baseline", "oracle_check")},
        **sub,
        "setup": {"selfcheck_failures_all_ranks": ds["selfcheck_failures_all_ranks"], "all_ok": ok},
    }
    return line, ok


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    N = world
    # the CPU baseline's OpenMP settings (reference run.sh:41,618-619), before any OpenMP runtime initialises
    os.environ.setdefault("OMP_PROC_BIND", "true")
    os.environ.setdefault("OMP_PLACES", "cores")
    os.environ.setdefault("OMP_DYNAMIC", "false")

    import numpy as np
    import torch
    import spmm_amd as S
    from spmm_amd import sharding
    from spmm_amd.datasets import CONFIG2_LINE, CONFIG4_LINE

    if not torch.cuda.is_available():
        print("error: no HIP device visible (bench.py measures the GPU engine; there is no CPU path)", file=sys.stderr)
        sys.exit(3)
    single = {"pipeline": run_pipeline, "medium-sample": run_medium_sample, "twins": run_twins}
    if args.workload in single:
        if N != 1:
            print(f"error: --workload {args.workload} runs on one GPU", file=sys.stderr)
            sys.exit(2)
        torch.cuda.set_device(0)
        if args.workload == "pipeline" and args.dtype == "f64" and "--dtype" not in sys.argv:
            args.dtype = "f32"                       # the reference pipeline's configuration
        sys.exit(single[args.workload](args, torch, S, np))

    dist = None
    ndev = torch.cuda.device_count()
    dev_index = local_rank % ndev if args.dist_backend == "gloo" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if N > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            dist.init_process_group(backend="gloo")
    ctx = Ctx(args, N, rank, dist, dev, dev_index, torch, S, np, sharding)

    if args.workload == "dataset":
        line, ok_all = run_dataset_line(ctx)
    else:
        gen = args.gen or (CONFIG4_LINE if args.workload == "config4" else CONFIG2_LINE)
        line, ok_all = measure_line(ctx, gen, args.scaling, args.workload, cpu=(args.workload == "config2"),
                                    e2e=(args.workload == "config2"), multi=True, dump=args.dump_c)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if not ok_all:
        print("error: self-check failed (C not finite, outside the normwise bound, or not bit-exact against the "
              "oracle on an exact row)", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
