#!/usr/bin/env python3
"""bench.py -- headline benchmark: CSR SpMM C = A*B, K=32, fp64, synthetic matrix, MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; N>1 is launched by torch.distributed.run,
one rank per GPU.  One "step" = one SpMM over the rank's row shard, inputs resident in HBM.  Rank 0 prints ONE
JSON line.

Workload (BASELINE.json configs[1]): generator line
    1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14
(1M x 1M, avg 20 nnz/row, normal row lengths, bw 0.3, skew 100, neighbours 0.95, cross-row similarity 0.5,
seed 14), A values seeded uniform [0.5, 1.5), B seeded uniform [0, 1), K = 32, fp64.
Multi-GPU (weak scaling): the global matrix is N x that shape -- N*1M rows and columns, bw scaled by 1/N so each
row keeps the same absolute column window -- split into N nnz-balanced row ranges with the reference partitioner
(loop_partitioner_balance_prefix_sums).  B is broadcast from rank 0 over RCCL once at setup; C stays sharded.
Each rank's shard is statistically the single-GPU workload.

JSON extras: "roofline" for the SpMM kernel (algorithmic bytes per launch / HIP-event-timed launch duration on the
launch stream), "cpu_baseline" (the reference kernel compiled from its sources, oracle/_ref, timed on this host
at N=1 on the same matrix, bounded number of calls), "hbm_gbs_alg".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "spmm-research_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
GEN_LINE = "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--gen", default=GEN_LINE, help="11-field generator line of the per-GPU workload")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="budget of timed CPU-baseline calls")
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "pmc_latest.json"),
                    help="per-launch HBM traffic collected by tools/collect_pmc.py (optional)")
    return ap.parse_args()


def engine_sha256() -> str:
    """Fingerprint of the engine build: its device/host sources and the Makefile (flags), so PMC numbers collected for
    one engine version stay attached to it across rebuilds (the .so bytes themselves are not reproducible: hipcc
    embeds build paths)."""
    import hashlib
    h = hashlib.sha256()
    pkg = ROOT / "spmm-research_amd"
    for f in (pkg / "csrc" / "spmm_engine.hip", pkg / "csrc" / "spmm_kernels.hpp", ROOT / "include" / "spmm_hip.h",
              pkg / "Makefile"):
        h.update(f.read_bytes())
    return h.hexdigest()


def cpu_baseline(A, k: int, budget_s: float) -> dict | None:
    """Reference compute_csr (oracle/_ref, compiled from /root/reference's sources) on this host, same matrix."""
    import numpy as np
    from oracle import oracle as O
    vt = "d"
    kind = "reference" if O.ref_available(vt) else "port"
    cores = min(16, len(os.sched_getaffinity(0)))
    x = O.drand48(42, A.ncols * k)
    vals = A.values.copy()
    if kind == "reference":
        L = O.ref_lib(vt)
        L.ref_set_threads(cores)
        y = np.zeros(A.m * k, np.float64)
        mf = L.ref_create(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k)
        call = lambda: L.ref_run(mf, x, y, k)  # noqa: E731
    else:
        call = lambda: O.spmm(A.row_ptr, A.col_idx, vals, A.ncols, x, k, cores)  # noqa: E731
    call()  # warm-up (the reference harness does 100; bounded here)
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 3 or (time.perf_counter() < t_end and len(times) < 100):
        t0 = time.perf_counter()
        call()
        times.append(time.perf_counter() - t0)
    times.sort()
    t = times[len(times) // 2]
    gf = 2.0 * A.nnz * k / t / 1e9
    return {"value": round(gf, 3), "unit": "GFLOP/s", "cores": cores, "kind": kind,
            "sample": f"full matrix (same A, B as the GPU run), 1 warm-up + {len(times)} timed calls, median "
                      f"{t * 1e3:.1f} ms/call, {cores} OpenMP threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    N = world

    import numpy as np
    import torch
    import spmm_amd as S

    dist = None
    if N > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    K = args.k
    tdtype = torch.float64 if args.dtype == "f64" else torch.float32
    npdtype = np.float64 if args.dtype == "f64" else np.float32

    # ---- global matrix: N stacked copies of the per-GPU shape, nnz-balanced row split (a8 partitioner)
    from spmm_amd import sharding
    t0 = time.perf_counter()
    p = sharding.weak_scaled_params(args.gen, N)
    sh = sharding.make_shard(p, N, rank)
    A = sh.a
    t_gen = time.perf_counter() - t0

    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdtype), A.m, p.nr_cols, A.nnz, K, local_rank)

    # ---- B (row-major [ncols][K]) resident in HBM, identical on every rank: rank 0 draws it, RCCL broadcast
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    B = torch.rand((p.nr_cols, K), generator=g, device=dev, dtype=tdtype) if rank == 0 else \
        torch.empty((p.nr_cols, K), device=dev, dtype=tdtype)
    t_bcast = 0.0
    if dist is not None:
        torch.cuda.synchronize()
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
    if dist is not None:
        tt = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_max_ms = float(tt[0]), float(tt[1])
        nn = torch.tensor([A.nnz], device=dev, dtype=torch.int64)
        dist.all_reduce(nn)
        nnz_total = int(nn[0])
    else:
        kern_max_ms, nnz_total = kern_ms, A.nnz

    # cheap self-consistency: C is finite and not all zero (parity proper lives in tests/ and smoke())
    csum = float(C.sum())
    ok = bool(np.isfinite(csum))

    flops_step = 2.0 * nnz_total * K
    gflops = flops_step * args.steps / elapsed / 1e9
    s = 8 if args.dtype == "f64" else 4
    # B's compulsory term: at N=1 all ncols rows of B (SURVEY §8d formula); at N>1 the rank's shard can only touch
    # the B rows of the columns it holds, so count those (the same formula with ncols = distinct columns)
    ncols_eff = p.nr_cols if N == 1 else int(np.unique(A.col_idx).size)
    bytes_launch = S.bytes_alg(A.m, ncols_eff, A.nnz, K, S.F64 if s == 8 else S.F32)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    # PMC traffic of THIS workload and THIS engine build (tools/collect_pmc.py, separate rocprofv3 --pmc passes)
    traffic = None
    try:
        pm = json.loads(Path(args.pmc_json).read_text())
        if (pm.get("workload") == args.gen and pm.get("k") == K and pm.get("dtype") == args.dtype and N == 1
                and pm.get("nnz") == A.nnz and pm.get("engine_sha256") == engine_sha256()):
            traffic = pm.get("hbm_bytes_per_launch")
    except Exception:
        pass

    cpu = None
    if rank == 0 and N == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(A, K, args.cpu_seconds)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "unit": "GFLOP/s", "cores": 0, "kind": "reference", "sample": f"failed: {e}"}

    if rank == 0:
        line = {
            "metric": "GFLOP/s + achieved HBM GB/s, synthetic medium dataset, CSR SpMM K=32 fp64",
            "value": round(gflops, 3),
            "unit": "GFLOP/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.dtype == "f64" else "f32",
            "data": "synthetic (own generator, seeded; A values U[0.5,1.5), B U[0,1))",
            "config": {"workload": f"csr_spmm gen='{args.gen}' x{N} rows/cols, K={K}",
                       "nnz_per_gpu": A.nnz, "nnz_total": nnz_total, "rows_total": int(p.nr_rows),
                       "k": K, "parallelism": f"row-shard{N}"},
            "hbm_gbs_alg": round(achieved, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         # PMC bytes per launch moved in the measured launch time: what the L2-miss stream actually
                         # sustains (the B gather re-fetches rows beyond L2)
                         "traffic_gbs": None if traffic is None else round(traffic / (kern_ms * 1e-3) / 1e9, 1),
                         "bytes_alg_per_launch": bytes_launch, "kernel_ms_per_launch": round(kern_ms, 5),
                         "kernel_ms_max_over_ranks": round(kern_max_ms, 5)},
            "cpu_baseline": cpu,
            "setup": {"gen_s": round(t_gen, 2), "bcast_B_s": round(t_bcast, 4), "finite": ok},
        }
        print(json.dumps(line), flush=True)
    mf.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
