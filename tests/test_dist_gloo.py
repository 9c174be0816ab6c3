"""Multi-rank path on CPU: world_size 2 (and 3) over gloo, strong and weak splits.

Each rank builds its nnz-balanced shard (reference partitioner loop_partitioner_balance_prefix_sums,
lib/parallel_util.h:141-165) -- of ONE global matrix (strong, config 4's shape: gamma rows, heavy skew) or of N
stacked copies (weak) -- receives B by broadcast from rank 0, computes its C rows (the CPU oracle stands in for the
GPU kernel: the sharding/communication logic is what is under test here; tests/test_gpu_configs.py runs the same
shards through the HIP engine), and the all-gathered C must equal the oracle on the whole matrix bit for bit.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
GEN_WEAK = "6000 5000 12 4 normal random 0.3 50 0.95 0.5 14"
# config 4 in miniature: a large-dataset line shape (avg 20, skew 10^4) with gamma row lengths
GEN_STRONG = "17189 17189 20 6.6667 gamma random 0.3 10000 0.95 0.5 14"
K = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, gen, mode):
    sys.path.insert(0, str(ROOT / "spmm-research_amd"))
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from spmm_amd import sharding
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = sharding.weak_scaled_params(gen, world) if mode == "weak" else sharding.strong_params(gen)
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
    assert counts[rank] == sh.r1 - sh.r0
    c_all = sharding.allgather_rows(dist, torch.from_numpy(np.ascontiguousarray(c_local)), counts)
    # per-rank scalars (bench.py's max-over-ranks kernel time, slowest rank's bytes, self-check flags)
    sc = sharding.gather_scalars(dist, [float(rank), float(counts[rank])], torch.device("cpu"))
    assert [v[0] for v in sc] == list(range(world)) and [v[1] for v in sc] == [float(c) for c in counts]
    if rank == 0:
        np.save(Path(outdir) / "c_all.npy", c_all.numpy())
        np.save(Path(outdir) / "x_col.npy", x_col)
        np.save(Path(outdir) / "meta.npy", np.array([sh.nnz_global, sh.m_global, sh.ncols_global]))
    dist.barrier()
    dist.destroy_process_group()


# world 8: the driver's 8-GPU node, rehearsed on CPU ranks (config 4's shape in miniature, and the weak split that
# bench.py runs by default at N > 1)
@pytest.mark.parametrize("mode,gen,world", [("weak", GEN_WEAK, 2), ("weak", GEN_WEAK, 3), ("weak", GEN_WEAK, 8),
                                            ("strong", GEN_STRONG, 2), ("strong", GEN_STRONG, 3),
                                            ("strong", GEN_STRONG, 8)])
def test_sharded_equals_whole(tmp_path, mode, gen, world):
    import spmm_amd as S
    from spmm_amd import sharding
    from oracle import oracle as O
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), gen, mode), nprocs=world, join=True)
    c_all = np.load(tmp_path / "c_all.npy")
    x_col = np.load(tmp_path / "x_col.npy")
    nnz, m, n = np.load(tmp_path / "meta.npy")
    p = sharding.weak_scaled_params(gen, world) if mode == "weak" else sharding.strong_params(gen)
    A = S.generate(p)
    assert (A.nnz, A.m, A.ncols) == (nnz, m, n)
    want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x_col, K)
    assert np.array_equal(c_all.view(np.int64), want.view(np.int64))


def test_strong_split_is_reference_partition():
    """The strong split of one global matrix: rank boundaries are the reference partitioner's, every row once."""
    import spmm_amd as S
    from spmm_amd import sharding
    from oracle import oracle as O
    p = sharding.strong_params(GEN_STRONG)
    A = S.generate(p)
    for world in (2, 4, 8):
        bounds = sharding.shard_bounds(p, world)
        assert bounds[0][0] == 0 and bounds[-1][1] == A.m
        for w in range(world):
            assert bounds[w] == O.partition(A.row_ptr, A.nnz, world, w)
            if w:
                assert bounds[w][0] == bounds[w - 1][1]
            sh = sharding.make_shard(p, world, w)
            lo, hi = A.row_ptr[bounds[w][0]], A.row_ptr[bounds[w][1]]
            assert np.array_equal(sh.a.col_idx, A.col_idx[lo:hi])
            assert np.array_equal(sh.a.values.view(np.int64), A.values[lo:hi].view(np.int64))
        assert sharding.imbalance(p, world) >= 1.0


def test_weak_scaled_shards_statistically_equal():
    import spmm_amd as S
    from spmm_amd import sharding
    one = S.features(S.generate(S.gen_params(GEN_WEAK)))
    p = sharding.weak_scaled_params(GEN_WEAK, 4)
    for r in range(4):
        sh = sharding.make_shard(p, 4, r)
        assert abs(sh.a.nnz - one["nr_nzeros"]) / one["nr_nzeros"] < 0.02
        assert abs(sh.a.m - one["nr_rows"]) / one["nr_rows"] < 0.02
    assert sharding.imbalance(p, 4) < 1.01


def test_bench_refuses_world_mismatch_on_cpu():
    """`bench.py --gpus 2` without torchrun starts its own ranks; on a box without a GPU every rank fails loudly
    (no silent one-GPU record); a WORLD_SIZE that differs from --gpus is refused."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout
