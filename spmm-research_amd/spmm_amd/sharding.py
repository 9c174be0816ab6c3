"""Row sharding of one CSR SpMM across ranks (one process per GPU), SURVEY.md §8e.

* Partition: contiguous nnz-balanced row ranges, the reference's loop_partitioner_balance_prefix_sums
  (lib/parallel_util.h:141-165) applied at GPU granularity (``partition_rows``).
* Data: each rank holds its rows' CSR slice (row_ptr rebased to 0, global column ids) -- generated directly for
  synthetic matrices (``spmm_host_generate_rows``), so no rank ever materialises the whole matrix.
* B: replicated; rank 0 owns it and ``broadcast_b`` sends it over the process group (RCCL over xGMI for the
  "nccl" backend on GPUs, gloo on CPU) once at setup.
* C: stays sharded during the timed steps; ``allgather_rows`` assembles it (variable row counts, padded
  all_gather) for validation only.

Strong scaling (bench.py default, config 4): ONE global matrix (the generator line as given) split N ways -- the
same problem at every N.  Weak scaling (bench.py --scaling weak): the global problem for N ranks is N stacked
copies of the single-GPU shape -- N*m rows, N*ncols columns, bw/N so each row keeps the same absolute column
window -- so every shard is statistically the one-GPU workload.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import CSR, gen_params, generate_row_ptr, generate_rows, partition_rows


@dataclass
class Shard:
    rank: int
    world: int
    r0: int
    r1: int
    a: CSR               # rows [r0, r1) with global column ids
    nnz_global: int
    m_global: int
    ncols_global: int


def weak_scaled_params(gen_line: str, world: int):
    """N x the single-GPU generator shape (rows, cols scaled; bw scaled down to keep the absolute window)."""
    p = gen_params(gen_line)
    p.nr_rows = p.nr_rows * world
    p.nr_cols = p.nr_cols * world
    p.bw = p.bw / world
    return p


def strong_params(gen_line: str):
    """The global matrix of a strong-scaling run: the generator line unchanged at every N."""
    return gen_params(gen_line)


def make_shard(params, world: int, rank: int) -> Shard:
    rp = generate_row_ptr(params)
    nnz = int(rp[-1])
    r0, r1 = partition_rows(rp, nnz, world, rank)
    a = generate_rows(params, r0, r1)
    return Shard(rank, world, r0, r1, a, nnz, int(params.nr_rows), int(params.nr_cols))


def shard_bounds(params, world: int) -> list[tuple[int, int]]:
    rp = generate_row_ptr(params)
    nnz = int(rp[-1])
    return [partition_rows(rp, nnz, world, w) for w in range(world)]


def _host_staged(dist, t) -> bool:
    """gloo (the CPU / shared-GPU test backend) runs the collectives below on host copies of device tensors."""
    return t.is_cuda and dist.get_backend() == "gloo"


def broadcast_b(dist, b, src: int = 0) -> None:
    """Replicate B (any torch tensor on the group's device) from `src` -- one collective, setup only."""
    if _host_staged(dist, b):
        h = b.cpu()
        dist.broadcast(h, src=src)
        b.copy_(h)
        return
    dist.broadcast(b, src=src)


def allgather_rows(dist, c_local, counts: list[int]):
    """Variable-count all-gather of row shards (torch tensors [rows, K]); returns the concatenated [sum, K]."""
    import torch
    world = len(counts)
    mx = max(counts) if counts else 0
    k = c_local.shape[1]
    staged = _host_staged(dist, c_local)
    dev = torch.device("cpu") if staged else c_local.device
    pad = torch.zeros((max(mx, 1), k), dtype=c_local.dtype, device=dev)
    n = counts[dist.get_rank()]
    pad[:n] = c_local[:n].to(dev)
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    out = torch.cat([bufs[w][: counts[w]] for w in range(world)], dim=0)
    return out.to(c_local.device) if staged else out


def gather_scalars(dist, vals: list[float], device) -> list[list[float]]:
    """Every rank's small vector of floats, on every rank (timings, byte counts, flags): [rank][i]."""
    import torch
    world = dist.get_world_size()
    dev = torch.device("cpu") if dist.get_backend() == "gloo" else device
    t = torch.zeros((world, len(vals)), dtype=torch.float64, device=dev)
    t[dist.get_rank()] = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return t.cpu().tolist()


def imbalance(params, world: int) -> float:
    """max / mean nonzeros per rank of the partition (1.0 = perfect); giant rows cap it."""
    rp = generate_row_ptr(params)
    nnz = int(rp[-1])
    per = [int(rp[e] - rp[s]) for s, e in (partition_rows(rp, nnz, world, w) for w in range(world))]
    return max(per) / (sum(per) / world) if sum(per) else 1.0
