"""Multi-rank path on CPU: world_size 2 (and 3) over gloo.  Each rank builds its nnz-balanced shard of the weak-scaled
global matrix, receives B by broadcast from rank 0, computes its C rows (with the CPU oracle standing in for the
GPU kernel -- the sharding/communication logic is what is under test), and the all-gathered C must equal the
oracle on the whole matrix bit for bit."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
GEN = "6000 5000 12 4 normal random 0.3 50 0.95 0.5 14"
K = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT / "spmm-research_amd"))
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from spmm_amd import sharding
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = sharding.weak_scaled_params(GEN, world)
    sh = sharding.make_shard(p, world, rank)
    # B row-major [ncols][K], drawn on rank 0 only, replicated by broadcast
    if rank == 0:
        b = torch.from_numpy(O.drand48(42, sh.ncols_global * K).reshape(sh.ncols_global, K))
    else:
        b = torch.empty((sh.ncols_global, K), dtype=torch.float64)
    sharding.broadcast_b(dist, b)
    x_col = np.ascontiguousarray(b.numpy().T).ravel()
    c_local = O.spmm(sh.a.row_ptr, sh.a.col_idx, sh.a.values, sh.ncols_global, x_col, K)
    counts = [e - s for s, e in sharding.shard_bounds(p, world)]
    c_all = sharding.allgather_rows(dist, torch.from_numpy(np.ascontiguousarray(c_local)), counts)
    if rank == 0:
        np.save(Path(outdir) / "c_all.npy", c_all.numpy())
        np.save(Path(outdir) / "x_col.npy", x_col)
        np.save(Path(outdir) / "meta.npy", np.array([sh.nnz_global, sh.m_global, sh.ncols_global]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_whole(tmp_path, world):
    import spmm_amd as S
    from spmm_amd import sharding
    from oracle import oracle as O
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    c_all = np.load(tmp_path / "c_all.npy")
    x_col = np.load(tmp_path / "x_col.npy")
    nnz, m, n = np.load(tmp_path / "meta.npy")
    p = sharding.weak_scaled_params(GEN, world)
    A = S.generate(p)
    assert (A.nnz, A.m, A.ncols) == (nnz, m, n)
    want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x_col, K)
    assert np.array_equal(c_all.view(np.int64), want.view(np.int64))


def test_weak_scaled_shards_statistically_equal():
    import spmm_amd as S
    from spmm_amd import sharding
    one = S.features(S.generate(S.gen_params(GEN)))
    p = sharding.weak_scaled_params(GEN, 4)
    for r in range(4):
        sh = sharding.make_shard(p, 4, r)
        assert abs(sh.a.nnz - one["nr_nzeros"]) / one["nr_nzeros"] < 0.02
        assert abs(sh.a.m - one["nr_rows"]) / one["nr_rows"] < 0.02
    assert sharding.imbalance(p, 4) < 1.01
