#!/usr/bin/env python3
"""bench.py -- headline benchmark: CSR SpMM C = A*B, K=32, fp64, synthetic matrix, MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  N>1 runs one rank per GPU; when it is not
started by torch.distributed.run (no WORLD_SIZE in the environment) it starts torch.distributed.run itself as a
CHILD process (before anything touches the GPU) and exits with its status.  A world size that differs from --gpus
is an error (exit 2).  One "step" = one SpMM over the rank's row shard, inputs resident in HBM.  Rank 0 prints ONE
JSON line.

Workloads (--workload):
  config2   (default; BASELINE.json configs[1]) generator line
            1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14
            (1M x 1M, avg 20 nnz/row, normal row lengths, bw 0.3, skew 100, neighbours 0.95, cross-row similarity
            0.5, seed 14).
  config4    the largest avg-20 skew-10^4 line of synthetic_matrices_large_dataset.txt with
            gamma row lengths: 7477550 7477550 20 6.6667 gamma random 0.3 10000 0.95 0.5 14 (150 M nonzeros).
  medium-sample  (config 3) every --sample-stride-th line of synthetic_matrices_medium_dataset (N=1 only); value =
            aggregate GFLOP/s over the sample (sum of flops / sum of kernel time).
  pipeline   the sparse-attention pipeline consumer, fp32, n=512: K/Q/V = W x (DLMC-like 512 x 512
            attention weights, 70 % pruned), SDDMM over a band+random mask (band 16, 5 % dense), final SpMM;
            one step = the reference compute() step (pipeline_code_bench/sddmm_bench.cpp:918-937), HBM-resident,
            captured in a hipGraph; GFLOP/s by the reference formula (:978-983).  N=1 only.
A values: the generator's seeded U[0.5, 1.5).  B: drand48(seed 42), drawn on the host in the reference harness's
column-major layout [K][ncols] (the same x the CPU baseline multiplies), uploaded transposed to the engine's
row-major layout, resident in HBM.

Multi-GPU (--scaling, default strong): STRONG = one fixed global matrix (the workload's line) split into N
nnz-balanced row ranges with the reference partitioner loop_partitioner_balance_prefix_sums
(lib/parallel_util.h:141-165); the same matrix at every N, so the driver's 1/2/4/8 values form a strong-scaling
curve.  WEAK = N stacked copies of the line's shape (bw/N).  Each rank generates only its rows; B is broadcast from
rank 0 over RCCL once at setup (timed, reported); C stays sharded in the timed loop and is all-gathered once
afterwards (timed, reported).  Per-rank kernel time (HIP events on the launch stream), its max over ranks and the
nnz imbalance (max/mean) are reported.

Self-check (every rank, every run): 256 sampled rows of the rank's C against a host recomputation with numpy
(normwise 1e-10 fp64 / (n+1)*2^-24 fp32); a failure or a non-finite C exits non-zero.  Bit-exact parity against
the oracle lives in tests/ (the oracle is test infrastructure and only the cpu_baseline leg below uses it).

JSON extras: "roofline" for the SpMM kernel (algorithmic bytes per launch -- SURVEY §8d, one definition at every N:
the rank's rows and nonzeros with the global column count -- over the HIP-event-timed launch duration),
"cpu_baseline" (oracle/liboracle.so, the bit-pinned C restatement of the reference compute_csr, timed on this
host at N=1 on the same A and B: 100 warm-up calls like the reference harness, then timed calls, median),
"setup" (generation, B broadcast, C all-gather), "plugin_e2e" (N=1: the reference-contract call with host x / y:
H2D + transpose + kernel + D2H).
"""
from __future__ import annotations

import argparse
import json
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--workload", choices=["config2", "config4", "medium-sample", "pipeline"], default="config2")
    ap.add_argument("--pipe-m", type=int, default=512, help="pipeline: weight rows = mask size")
    ap.add_argument("--pipe-k", type=int, default=512, help="pipeline: weight columns (rows of x)")
    ap.add_argument("--pipe-n", type=int, default=512, help="pipeline: columns of x (NUM_COLS)")
    ap.add_argument("--pipe-density", type=float, default=0.3, help="pipeline: weight density (1 - pruning)")
    ap.add_argument("--pipe-mask-density", type=float, default=0.05)
    ap.add_argument("--pipe-band", type=int, default=16)
    ap.add_argument("--pipe-mode", type=int, default=0, help="pipeline: SDDMM flags (0 reference, 1 QK^T, |2 softmax)")
    ap.add_argument("--gen", default=None, help="override: 11-field generator line of the global matrix")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--sample-stride", type=int, default=160, help="medium-sample: every n-th dataset line")
    ap.add_argument("--sample-offset", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-warmup", type=int, default=100, help="CPU-baseline warm-up calls (reference harness: 100)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="budget of timed CPU-baseline calls")
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "pmc_latest.json"),
                    help="per-launch HBM traffic collected by tools/collect_pmc.py (optional)")
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
    for f in (pkg / "csrc" / "spmm_engine.hip", pkg / "csrc" / "spmm_kernels.hpp", ROOT / "include" / "spmm_hip.h",
              pkg / "Makefile"):
        h.update(f.read_bytes())
    return h.hexdigest()


def cpu_baseline(A, x_col, k: int, warmup: int, budget_s: float, dtype) -> dict:
    """The reference compute_csr (restated in oracle/spmm_oracle.c, bit-pinned against the reference build) on this
    host, same A and the same column-major x the GPU's B was made from."""
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
    return {"value": round(gf, 3), "unit": "GFLOP/s", "cores": threads, "kind": "port",
            "sample": (f"full matrix, same A and x (drand48 seed 42, column-major) as the GPU run; oracle/liboracle.so "
                       f"(C restatement of compute_csr, bit-identical to the reference build); {threads} OpenMP threads "
                       f"(OMP_PROC_BIND=true OMP_PLACES=cores OMP_DYNAMIC=false) on {model}; {warmup} warm-up calls "
                       f"({t_warm:.1f} s) + {len(times)} timed, median {t * 1e3:.1f} ms/call")}


def selfcheck(A, B_host_rowmajor, C_dev, k: int, dtype, nsample: int = 256, seed: int = 5) -> dict:
    """numpy recomputation of sampled rows (not the oracle; a sanity check of the run, parity is in tests/)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    m = A.m
    if m == 0:
        return {"rows": 0, "ok": True}
    deg = np.diff(A.row_ptr)
    rows = np.unique(np.concatenate([rng.choice(m, min(nsample, m), replace=False), [int(np.argmax(deg))]]))
    import torch
    got_all = C_dev[torch.from_numpy(rows).to(C_dev.device)].cpu().numpy().astype(np.float64)
    ok = True
    worst = 0.0
    for i, r in enumerate(rows):
        s, e = int(A.row_ptr[r]), int(A.row_ptr[r + 1])
        got = got_all[i]
        bv = B_host_rowmajor[A.col_idx[s:e]].astype(np.float64)
        av = A.values[s:e].astype(dtype).astype(np.float64)
        want = av @ bv if e > s else np.zeros(k)
        absdot = np.abs(av) @ np.abs(bv) if e > s else np.zeros(k)
        tol = 1e-10 if dtype == np.float64 else (e - s + 1) * 2.0 ** -24
        bound = tol * np.maximum(np.abs(want), absdot) + 1e-300
        err = np.abs(got - want) / bound
        worst = max(worst, float(err.max()) if len(err) else 0.0)
        ok = ok and bool(np.all(np.isfinite(got))) and bool(np.all(err <= 1.0 + 1e-9))
    return {"rows": int(len(rows)), "ok": ok, "max_err_over_bound": round(worst, 6)}


def run_medium_sample(args, torch, S, np):
    """config 3 at N=1: a strided sample of the medium dataset; aggregate GFLOP/s = sum(flops) / sum(kernel time)."""
    from spmm_amd.datasets import medium_dataset_lines
    lines = medium_dataset_lines()[args.sample_offset::args.sample_stride]
    dev = torch.device("cuda", 0)
    K = args.k
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    npdt = np.float64 if args.dtype == "f64" else np.float32
    stream = torch.cuda.current_stream(dev)
    tot_flops = tot_s = tot_bytes = 0.0
    fracs, bad = [], 0
    t_start = time.perf_counter()
    for i, line in enumerate(lines):
        A = S.generate(S.gen_params(line))
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdt), A.m, A.ncols, A.nnz, K, 0)
        x = S.drand48(42, A.ncols * K)
        Bh = np.ascontiguousarray(x.reshape(K, A.ncols).T).astype(npdt)
        B = torch.from_numpy(Bh).to(dev)
        C = torch.empty((max(A.m, 1), K), device=dev, dtype=tdt)
        for _ in range(args.warmup):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), K, stream.cuda_stream)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(args.steps):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), K, stream.cuda_stream)
        ev1.record(stream)
        torch.cuda.synchronize()
        t = ev0.elapsed_time(ev1) / args.steps * 1e-3
        chk = selfcheck(A, Bh, C, K, npdt, nsample=32)
        bad += 0 if chk["ok"] else 1
        b = S.bytes_alg(A.m, A.ncols, A.nnz, K, S.F64 if args.dtype == "f64" else S.F32)
        tot_flops += 2.0 * A.nnz * K
        tot_s += t
        tot_bytes += b
        fracs.append(b / t / 1e9 / HBM_PEAK_GBS)
        mf.close()
        del B, C
        print(f"[{i + 1}/{len(lines)}] {line}: {2.0 * A.nnz * K / t / 1e9:.1f} GFLOP/s frac {fracs[-1]:.3f}",
              file=sys.stderr, flush=True)
    elapsed = time.perf_counter() - t_start
    fr = sorted(fracs)
    line = {
        "metric": METRIC, "value": round(tot_flops / tot_s / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(tot_s / len(lines) * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (own generator, seeded; A values U[0.5,1.5), B drand48(42))",
        "config": {"workload": f"medium-sample: every {args.sample_stride}th line of synthetic_matrices_medium_dataset "
                               f"from {args.sample_offset} ({len(lines)} matrices), K={K}", "k": K,
                   "parallelism": "single-gpu"},
        "hbm_gbs_alg": round(tot_bytes / tot_s / 1e9, 2),
        "roofline": {"bound": "hbm", "achieved": round(tot_bytes / tot_s / 1e9, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(tot_bytes / tot_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                     "median_frac": round(fr[len(fr) // 2], 4), "p10_frac": round(fr[len(fr) // 10], 4),
                     "p90_frac": round(fr[(9 * len(fr)) // 10], 4)},
        "cpu_baseline": None,
        "setup": {"wall_s": round(elapsed, 1), "selfcheck_failures": bad},
    }
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
        "warmup": args.warmup, "ms_per_step": round(step_ms, 5), "higher_is_better": True, "scaling": "weak",
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
    if args.workload == "pipeline":
        if N != 1:
            print("error: --workload pipeline runs on one GPU", file=sys.stderr)
            sys.exit(2)
        torch.cuda.set_device(0)
        if args.dtype == "f64" and "--dtype" not in sys.argv:
            args.dtype = "f32"                       # the reference pipeline's configuration
        sys.exit(run_pipeline(args, torch, S, np))
    if args.workload == "medium-sample":
        if N != 1:
            print("error: --workload medium-sample runs on one GPU", file=sys.stderr)
            sys.exit(2)
        torch.cuda.set_device(0)
        sys.exit(run_medium_sample(args, torch, S, np))

    dist = None
    torch.cuda.set_device(local_rank)
    if N > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    K = args.k
    tdtype = torch.float64 if args.dtype == "f64" else torch.float32
    npdtype = np.float64 if args.dtype == "f64" else np.float32
    gen = args.gen or (CONFIG4_LINE if args.workload == "config4" else CONFIG2_LINE)
    scaling = args.scaling

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
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdtype), A.m, ncols, A.nnz, K, local_rank)
    t_plan = time.perf_counter() - t0

    # ---- B: drand48(42) column-major x on rank 0 (the reference harness convention), row-major in HBM, broadcast
    x_col = None
    if rank == 0:
        x_col = S.drand48(42, ncols * K)
        Bh = np.ascontiguousarray(x_col.reshape(K, ncols).T).astype(npdtype)
        B = torch.from_numpy(Bh).to(dev)
    else:
        B = torch.empty((ncols, K), device=dev, dtype=tdtype)
    t_bcast = 0.0
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
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
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)   # HIP events on the launch stream
    kern_all = [kern_ms]
    if dist is not None:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])
        kt = torch.zeros(N, device=dev, dtype=torch.float64)
        kt[rank] = kern_ms
        dist.all_reduce(kt)
        kern_all = [float(v) for v in kt.cpu()]
    kern_max_ms = max(kern_all)

    # ---- C all-gather, once, timed (validation / hand-back path, never inside the timed loop)
    t_gather = None
    if dist is not None:
        counts = [e - s for s, e in bounds]
        torch.cuda.synchronize()
        dist.barrier()
        tg = time.perf_counter()
        c_all = sharding.allgather_rows(dist, C, counts)
        torch.cuda.synchronize()
        t_gather = time.perf_counter() - tg
        del c_all

    # ---- self-check on every rank (B rows for the check: rank 0 has them on the host; others copy from HBM)
    Bh_chk = Bh if rank == 0 else B.cpu().numpy()
    chk = selfcheck(A, Bh_chk, C, K, npdtype)
    ok_local = chk["ok"]
    if dist is not None:
        okt = torch.tensor([0 if ok_local else 1], device=dev, dtype=torch.int32)
        dist.all_reduce(okt)
        ok_all = int(okt[0]) == 0
    else:
        ok_all = ok_local

    flops_step = 2.0 * nnz_total * K
    gflops = flops_step * args.steps / elapsed / 1e9
    s = 8 if args.dtype == "f64" else 4
    dt_code = S.F64 if s == 8 else S.F32
    bytes_launch = S.bytes_alg(A.m, ncols, A.nnz, K, dt_code)      # one definition at every N (rank's rows, all cols)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic = None
    try:
        pm = json.loads(Path(args.pmc_json).read_text())
        if (pm.get("workload") == gen and pm.get("k") == K and pm.get("dtype") == args.dtype and N == 1
                and pm.get("nnz") == A.nnz and pm.get("engine_sha256") == engine_sha256()):
            traffic = pm.get("hbm_bytes_per_launch")
    except Exception:
        pass

    # ---- plugin end to end (N=1): host x / y through the reference contract (H2D + transpose + kernel + D2H)
    e2e = None
    if N == 1 and args.workload == "config2":
        y = np.empty(A.m * K, npdtype)
        xh = x_col.astype(npdtype)
        mf.spmm(xh, y, K)
        te = []
        for _ in range(3):
            t1 = time.perf_counter()
            mf.spmm(xh, y, K)
            te.append(time.perf_counter() - t1)
        lt = mf.last_times()
        e2e = {"ms_per_call": round(sorted(te)[1] * 1e3, 3),
               "gflops": round(flops_step / sorted(te)[1] / 1e9, 2),
               "events_ms": {k_: round(v, 4) for k_, v in lt.items()},
               "note": "pageable host buffers; PCIe-inclusive, never the headline value"}
        del y, xh

    cpu = None
    if rank == 0 and N == 1 and args.workload == "config2" and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(A, x_col, K, args.cpu_warmup, args.cpu_seconds, npdtype)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "unit": "GFLOP/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(gflops, 3),
            "unit": "GFLOP/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (own generator, seeded; A values U[0.5,1.5), B drand48(42))",
            "config": {"workload": f"{args.workload}: csr_spmm gen='{gen}'"
                                   + (f" x{N} stacked (weak)" if scaling == "weak" and N > 1 else "")
                                   + f", K={K}",
                       "nnz_total": nnz_total, "rows_total": int(p.nr_rows), "cols": ncols, "k": K,
                       "nnz_per_rank": per_rank, "imbalance_max_over_mean": round(imbalance, 4),
                       "parallelism": f"row-shard{N}" if N > 1 else "single-gpu"},
            "hbm_gbs_alg": round(achieved, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_gbs": None if traffic is None else round(traffic / (kern_ms * 1e-3) / 1e9, 1),
                         "bytes_alg_per_launch": bytes_launch, "kernel_ms_per_launch": round(kern_ms, 5),
                         "kernel_ms_per_rank": [round(v, 5) for v in kern_all],
                         "kernel_ms_max_over_ranks": round(kern_max_ms, 5)},
            "cpu_baseline": cpu,
            "plugin_e2e": e2e,
            "setup": {"gen_s": round(t_gen, 2), "plan_s": round(t_plan, 2), "bcast_B_s": round(t_bcast, 4),
                      "allgather_C_s": None if t_gather is None else round(t_gather, 4),
                      "selfcheck": chk, "selfcheck_all_ranks_ok": ok_all},
        }
        print(json.dumps(line), flush=True)
    mf.close()
    if dist is not None:
        dist.destroy_process_group()
    if not ok_all:
        print("error: self-check failed (C not finite or outside the normwise bound)", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
