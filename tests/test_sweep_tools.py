"""Sweep tooling (CPU): the medium dataset regenerated from its recipe equals the published file (pinned hash)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))


def test_medium_dataset_lines_match_published_set():
    from spmm_amd.datasets import medium_dataset_lines, sorted_sha256, SHA256_SORTED
    L = medium_dataset_lines()
    assert len(L) == 16190 and len(set(L)) == 16190
    assert sorted_sha256(L) == SHA256_SORTED
    for line in L[:50] + L[-50:]:
        f = line.split()
        assert len(f) == 11 and f[4] == "normal" and f[5] == "random" and f[10] == "14"


def test_sample_parity_checks_exact_and_inexact_rows():
    """tools/sweep.py's per-record check: exact rows bit for bit against the oracle, the others (only they need the
    __float128 gold) normwise; a perturbed inexact row inside 1e-10 passes, one outside fails."""
    import numpy as np
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    import sweep
    A = S.generate(S.gen_params("3000 3000 20 6.6667 normal random 0.3 100 0.95 0.5 14"))
    k = 8
    B = torch.from_numpy(O.drand48(5, A.ncols * k).reshape(A.ncols, k))
    x_col = np.ascontiguousarray(B.numpy().T).ravel()
    C = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x_col, k)
    exact = np.ones(A.m, bool)
    exact[::7] = False
    Ct = torch.from_numpy(C.copy())
    r = sweep.sample_parity(S, O, A, B, Ct, k, 300, np.random.default_rng(0), np.float64, exact)
    assert r["bitexact_seq_rows"] and r["normwise_ok"] and r["long_rows_checked"] > 0
    Ct[::7] *= 1 + 1e-13                                # inexact rows, inside the bound
    r = sweep.sample_parity(S, O, A, B, Ct, k, 3000, np.random.default_rng(0), np.float64, exact)
    assert r["bitexact_seq_rows"] and r["normwise_ok"]
    Ct[::7] *= 1 + 1e-8                                 # outside
    r = sweep.sample_parity(S, O, A, B, Ct, k, 3000, np.random.default_rng(0), np.float64, exact)
    assert r["bitexact_seq_rows"] and not r["normwise_ok"]
    Ct[1] += 1e-300 if Ct[1, 0] == 0 else Ct[1, 0] * 1e-15   # an exact row one ulp-ish off
    r = sweep.sample_parity(S, O, A, B, Ct, k, 3000, np.random.default_rng(0), np.float64, exact)
    assert not r["bitexact_seq_rows"]


def test_sweep_where_filter_selects_the_matrix_core_classes():
    """tools/sweep.py --where (the final-build re-sweep of DESIGN §6.17): crs 0.95 and >= 20 nonzeros per row is one
    third of the cross-row-similarity grid times four of the six row-length classes, in interleave16 order."""
    import argparse
    import sweep
    a = argparse.Namespace(line=None, dataset="medium", order="interleave16", sort_by_size=False, offset=0, stride=1,
                           where="crs=0.95,min_avg=20")
    sel = sweep.dataset_index_lines(a)
    assert len(sel) == 3596
    assert all(float(l.split()[9]) == 0.95 and float(l.split()[2]) >= 20 for _, l in sel)
    a.where = ""
    full = sweep.dataset_index_lines(a)
    assert len(full) == 16190
    assert [i for i, _ in sel] == [i for i, l in full if float(l.split()[9]) == 0.95 and float(l.split()[2]) >= 20]


def test_pmc_busy_time_counts_overlap_once():
    """tools/pmc_dataset.py: a matrix-core launch overlaps kernels on two streams; its kernel time is the union of
    the dispatch intervals, not their sum."""
    import pmc_dataset as P
    assert P.busy_ns([(0, 10), (5, 20), (30, 40)]) == 30
    assert P.busy_ns([(0, 100), (10, 20)]) == 100
    disp = [(1, "spmm_mfma_tile_kernel<double>", {"ns": 100.0}, (0.0, 100.0)),
            (2, "mfma_range_kernel<double>", {"ns": 20.0}, (5.0, 25.0)),
            (3, "spmm_rows_kernel<double>", {"ns": 50.0}, (25.0, 75.0)),
            (4, "mfma_fixup_kernel<double>", {"ns": 4.0}, (104.0, 108.0)),
            (5, "at::FillFunctor", {"ns": 1.0}, (110.0, 111.0))]
    g = P.per_matrix(disp, 1)
    assert g[0]["ns"] == 174.0 and g[0]["busy_ns"] == 104.0


def test_sweep_done_pairs_and_changed_pairs(tmp_path):
    """tools/sweep_done_pairs.py lists the measured (line, K) pairs of A/B record files in the census pair format."""
    import json
    import subprocess
    rec = tmp_path / "r.jsonl"
    rec.write_text(json.dumps({"gen": "1 1 1", "k": 32, "ms": 1.0, "ms_base": 1.1}) + "\n" +
                   json.dumps({"gen": "2 2 2", "k": 128, "ms": 1.0}) + "\n")
    out = tmp_path / "done.txt"
    tool = Path(__file__).resolve().parents[1] / "tools" / "sweep_done_pairs.py"
    subprocess.run([sys.executable, str(tool), str(rec), "--out", str(out)], check=True, capture_output=True)
    assert out.read_text() == "32\t1 1 1\n"


def _gen(avg, bw):
    return f"1000 1000 {avg} 1 normal random {bw} 0 0.5 0.5 14"


def test_sweep_flag_selects_slow_same_plan_and_spread_batches(tmp_path):
    """tools/sweep_flag.py: a record > 1.3x the reference's same plan is flagged, a faster one or one whose plan
    changed (tiles) is not; a record whose batches disagree by > 1.25x is flagged on its own."""
    import json
    import subprocess
    plan = {"blocks": 10, "panel_k": 32, "windows": 1, "split_rows": 0, "tiles": 0, "dtype": "f64"}
    ref = [dict(gen=_gen(20, 0.05), k=128, ms=1.0, **plan), dict(gen=_gen(20, 0.3), k=128, ms=1.0, **plan),
           dict(gen=_gen(50, 0.05), k=32, ms=1.0, **plan)]
    new = [dict(gen=_gen(20, 0.05), k=128, ms=2.0, batches=[2.0, 2.0, 2.1], **plan),      # same plan, 2x: flagged
           dict(gen=_gen(20, 0.3), k=128, ms=0.9, batches=[0.9, 0.95, 0.9], **plan),       # faster: kept
           dict(gen=_gen(50, 0.05), k=32, ms=2.0, batches=[2.0, 2.0, 2.0], **{**plan, "tiles": 5}),   # tiles: kept
           dict(gen=_gen(5, 0.6), k=8, ms=1.0, batches=[1.0, 1.6, 1.1], **plan)]           # batch spread: flagged
    (tmp_path / "ref.jsonl").write_text("".join(json.dumps(r) + "\n" for r in ref))
    (tmp_path / "new.jsonl").write_text("".join(json.dumps(r) + "\n" for r in new))
    out = tmp_path / "pairs.txt"
    tool = Path(__file__).resolve().parents[1] / "tools" / "sweep_flag.py"
    subprocess.run([sys.executable, str(tool), str(tmp_path / "new.jsonl"), "--ref", str(tmp_path / "ref.jsonl"),
                    "--out", str(out)], check=True, capture_output=True)
    assert out.read_text().splitlines() == [f"8\t{_gen(5, 0.6)}", f"128\t{_gen(20, 0.05)}"]


def test_sweep_compare_speedups(tmp_path):
    """tools/sweep_compare.py: per-K geomean of old / new kernel time over the common (line, K) pairs."""
    import json
    import subprocess
    old = [dict(gen=_gen(20, 0.05), k=32, ms=2.0, nnz=20000, roofline_frac=0.1),
           dict(gen=_gen(500, 0.3), k=32, ms=1.0, nnz=500000, roofline_frac=0.2)]
    new = [dict(gen=_gen(20, 0.05), k=32, ms=1.0, nnz=20000, roofline_frac=0.2),
           dict(gen=_gen(500, 0.3), k=32, ms=1.0, nnz=500000, roofline_frac=0.2)]
    (tmp_path / "o.jsonl").write_text("".join(json.dumps(r) + "\n" for r in old))
    (tmp_path / "n.jsonl").write_text("".join(json.dumps(r) + "\n" for r in new))
    tool = Path(__file__).resolve().parents[1] / "tools" / "sweep_compare.py"
    r = subprocess.run([sys.executable, str(tool), str(tmp_path / "o.jsonl"), str(tmp_path / "n.jsonl")],
                       check=True, capture_output=True, text=True)
    row = [l for l in r.stdout.splitlines() if l.startswith("| 32 |")][0]
    assert "| 2 | 1.414 |" in row                               # sqrt(2 x 1)


def test_gpu_rwlock_writer_excludes_readers_and_is_not_starved(tmp_path):
    """tools/gpu_rwlock.py: readers share; a writer waits for the readers inside, and a reader arriving after the
    writer waits for it (writer preference) -- checked with three processes and a shared event log.  The arrival
    order is forced by events, not delays: W starts once R1 is inside, R2 once W holds the gate, and R1
    leaves only after R2 has started waiting."""
    import errno
    import fcntl
    import multiprocessing as mp
    import time
    from gpu_rwlock import GpuRWLock
    path, log = str(tmp_path / "gpu.lock"), tmp_path / "log.txt"
    ctx = mp.get_context("fork")
    r1_in, w_start, r2_wait = ctx.Event(), ctx.Event(), ctx.Event()

    def note(s):
        with open(log, "a") as f:
            f.write(f"{time.monotonic():.6f} {s}\n")

    def reader1():
        lk = GpuRWLock(path)
        with lk.shared():
            note("R1 in")
            r1_in.set()
            assert r2_wait.wait(20)
            time.sleep(0.2)               # R2 is blocked at the gate by now; the order below holds either way
            note("R1 out")

    def writer():
        assert r1_in.wait(20)
        lk = GpuRWLock(path)
        w_start.set()
        with lk.exclusive():
            note("W in")
            time.sleep(0.1)
            note("W out")

    def reader2():
        assert w_start.wait(20)
        gate = open(path + ".gate", "a+")
        while True:                        # wait until the writer holds the gate
            try:
                fcntl.flock(gate, fcntl.LOCK_EX | fcntl.LOCK_NB)
                fcntl.flock(gate, fcntl.LOCK_UN)
                time.sleep(0.01)
            except OSError as e:
                assert e.errno in (errno.EWOULDBLOCK, errno.EAGAIN)
                break
        lk = GpuRWLock(path)
        r2_wait.set()
        with lk.shared():
            note("R2 in")
            note("R2 out")

    ps = [ctx.Process(target=reader1), ctx.Process(target=writer), ctx.Process(target=reader2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ev = [l.split(" ", 1)[1] for l in sorted(log.read_text().splitlines())]
    assert ev == ["R1 in", "R1 out", "W in", "W out", "R2 in", "R2 out"]
