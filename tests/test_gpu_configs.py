"""GPU parity on the BASELINE configs' own workloads (configs 3, 4 and 5), through the C ABI (-m gpu).

* Config 3 (synthetic_matrices_medium_dataset, K in {1, 8, 32, 128}, fp64): one line of every avg class
  {5,10,20,50,100,500} x bw {0.05, 0.6}, drawn with a fixed seed from the dataset's own lines (tools-free restatement
  of its recipe, spmm_amd.datasets), plus the dense-band line 39120 x 500 bw 0.05.
* Config 5 (validation twins, reference config.sh:283-339): every twin up to 40 M nonzeros (44 of 53), fp32 AND
  fp64, K=32.
* Config 4 (large dataset, gamma rows, nnz-balanced split over 8 GPUs): the 8 shards of the reference partitioner
  (lib/parallel_util.h:141-165) run one after another on this GPU; concatenated they must equal the whole-matrix
  run on every row both runs compute exactly, and a row sample of every shard must match the oracle.  Once in
  miniature (962,627 rows) and once at full size (CONFIG4_LINE, 7,477,550 rows, 150 M nonzeros).
Every check: rows the engine reports exact are bit-identical to the oracle (compute_csr restated,
spmm_kernel_csr.cpp:70-96); all sampled rows within 1e-10 normwise (fp64) / (n+1)*2^-24 (fp32).
"""
import random

import numpy as np
import pytest

from gpu_check import check_rows, run_device, sample_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, S, O


def medium_lines():
    from spmm_amd.datasets import medium_dataset_lines
    rng = random.Random(11)
    L = medium_dataset_lines()
    out = []
    for avg in (5, 10, 20, 50, 100, 500):
        for bw in (0.05, 0.6):
            cand = [l for l in L if float(l.split()[2]) == avg and float(l.split()[6]) == bw
                    and int(l.split()[0]) <= 1_000_000 and int(l.split()[0]) * avg <= 2e7]
            out.append(rng.choice(cand))
    out.append("39120 39120 500 166.6667 normal random 0.05 0 0.05 0.95 14")
    assert all(l in set(L) for l in out)
    return out


MEDIUM = medium_lines()


@pytest.mark.parametrize("line", MEDIUM, ids=[l.replace(" ", "_")[:48] for l in MEDIUM])
def test_config3_medium_lines(env, line):
    torch, S, O = env
    A = S.generate(S.gen_params(line))
    rows = sample_rows(A, 1500)
    for k in (1, 8, 32, 128):
        B, C, inf, ex = run_device(torch, S, A, k)
        assert np.isfinite(C).all()
        n_ex, n_in = check_rows(O, A, B, C, ex, rows)
        assert n_ex + n_in == len(rows)


def twin_names(max_nnz=4.0e7):
    """Every validation twin up to max_nnz nonzeros (44 of the 53 lines; the 9 larger ones -- up to kmer_V2a's
    117 M nonzeros -- run in `bench.py --workload twins`)."""
    from spmm_amd.datasets import twins
    out = []
    for name, line in twins().items():
        f = line.split()
        if int(f[0]) * float(f[2]) <= max_nnz:
            out.append(name)
    return out


TWINS = twin_names()


@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("name", TWINS)
def test_config5_twins(env, name, dtype):
    torch, S, O = env
    from spmm_amd.datasets import twins
    A = S.generate(S.gen_params(twins()[name]))
    B, C, inf, ex = run_device(torch, S, A, 32, dtype=dtype)
    assert np.isfinite(C).all()
    check_rows(O, A, B, C, ex, sample_rows(A, 2000), dtype=dtype)


def _split_8_ways(env, line, nsample):
    torch, S, O = env
    from spmm_amd import sharding
    p = sharding.strong_params(line)
    A = S.generate(p)
    k = 32
    B, C_whole, _, ex_whole = run_device(torch, S, A, k)
    bounds = sharding.shard_bounds(p, 8)
    assert bounds[0][0] == 0 and bounds[-1][1] == A.m
    for w, (r0, r1) in enumerate(bounds):
        assert (r0, r1) == O.partition(A.row_ptr, A.nnz, 8, w)
    per = [int(A.row_ptr[e] - A.row_ptr[s]) for s, e in bounds]
    C_cat = np.empty_like(C_whole)
    ex_cat = np.zeros(A.m, bool)
    dev = torch.device("cuda", 0)
    Bd = torch.from_numpy(B).to(dev)
    for w, (r0, r1) in enumerate(bounds):
        sh = sharding.make_shard(p, 8, w)
        assert sh.a.m == r1 - r0 and sh.a.nnz == per[w]
        Cd = torch.full((max(sh.a.m, 1), k), float("nan"), device=dev, dtype=torch.float64)
        mf = S.csr_to_format(sh.a.row_ptr, sh.a.col_idx, sh.a.values, sh.a.m, A.ncols, sh.a.nnz, k, 0)
        mf.spmm_device(Bd.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ex_cat[r0:r1] = mf.exact_rows()
        mf.close()
        C_cat[r0:r1] = Cd.cpu().numpy()[:sh.a.m]
        # every shard: oracle on a row sample of the shard (rows renumbered to the global matrix)
        rows = r0 + sample_rows(sh.a, nsample)
        check_rows(O, A, B, C_cat, ex_cat, rows)
    both = ex_whole & ex_cat
    assert both.mean() > 0.99
    assert np.array_equal(C_cat[both].view(np.int64), C_whole[both].view(np.int64))
    assert np.isfinite(C_cat).all()
    return max(per) / (sum(per) / 8)


def test_config4_gamma_split_8_ways_small(env):
    imb = _split_8_ways(env, "962627 962627 20 6.6667 gamma random 0.3 10000 0.95 0.5 14", 500)
    assert imb < 1.05


def test_config4_gamma_split_8_ways_full(env):
    from spmm_amd.datasets import CONFIG4_LINE
    imb = _split_8_ways(env, CONFIG4_LINE, 300)
    assert imb < 1.05


def test_run_device_colmajor_invalidates_upload_cache(env, monkeypatch):
    """run(x) -> run_device(col-major B2) -> run(x) with SPMM_HIP_ASSUME_X_UNCHANGED=1 must multiply x,
    not the B2 the device path left in the handle's internal buffer."""
    torch, S, O = env
    A = S.generate(S.gen_params("20000 20000 20 6.6667 normal random 0.3 100 0.95 0.5 14"))
    k = 8
    monkeypatch.setenv("SPMM_HIP_ASSUME_X_UNCHANGED", "1")
    mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
    x = O.drand48(42, A.ncols * k)
    y1 = np.zeros(A.m * k)
    mf.spmm(x, y1, k)
    dev = torch.device("cuda", 0)
    B2 = torch.from_numpy(O.drand48(7, A.ncols * k)).to(dev)       # column-major [k][ncols]
    C2 = torch.empty((A.m, k), dtype=torch.float64, device=dev)
    mf.spmm_device(B2.data_ptr(), S.B_COL_MAJOR, C2.data_ptr(), k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    y2 = np.zeros(A.m * k)
    mf.spmm(x, y2, k)
    mf.close()
    assert np.array_equal(y1.view(np.int64), y2.view(np.int64))
    assert not np.array_equal(C2.cpu().numpy().ravel().view(np.int64), y1.view(np.int64))
