"""bench.py on the GPU (-m gpu): the N>1 path before the driver's 8-GPU run, and the dataset record.

* `bench.py --gpus 2 --dist-backend gloo`: two ranks (self-spawned torch.distributed.run) share cuda:0 -- the
  strong split of config 2 by the reference partitioner (lib/parallel_util.h:141-165), B broadcast, per-rank HIP-event
  timing (value from the slowest rank), C all-gathered once, every rank self-checked.  The gathered C must
  be bit-equal to the one-rank run on every sampled row both runs compute exactly.
  The same run drives the in-process multi-GPU handle of the C ABI (spmm_hip_create_multi, shards on repeated
  device 0): peer B broadcast, spmm_hip_run_sharded timed, C gathered and self-checked.
* `--workload medium-sample` on a small stride: the dataset record's fields (aggregate, fractions, CPU baseline).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _bench(args, timeout=600):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_share_one_gpu(tmp_path):
    c2, c1 = tmp_path / "c2.npz", tmp_path / "c1.npz"
    two = _bench(["--gpus", "2", "--workload", "config2", "--scaling", "strong", "--dist-backend", "gloo",
                  "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--dump-c", str(c2)])
    assert two["n_gpus"] == 2 and two["config"]["dist_backend"] == "gloo"
    assert sum(two["config"]["nnz_per_rank"]) == two["config"]["nnz_total"]
    assert two["setup"]["selfcheck_all_ranks_ok"] is True
    rl = two["roofline"]
    assert len(rl["kernel_ms_per_rank"]) == 2
    assert rl["kernel_ms_per_launch"] == max(rl["kernel_ms_per_rank"]) == two["ms_per_step"]
    assert abs(two["value"] - 2 * two["config"]["nnz_total"] * 32 / (two["ms_per_step"] * 1e-3) / 1e9) < 1e-3 * two["value"]
    assert two["wall_ms_per_step"] >= 0.9 * two["ms_per_step"]
    assert two["setup"]["allgather_C_s"] is not None and two["dataset"] is None
    # the in-process multi-GPU handle (spmm_hip_create_multi) on repeated devices: peer broadcast, sharded runs
    mh = two["multi_handle"]
    assert mh is not None and "error" not in mh, mh
    assert mh["devices"] == [0, 0] and mh["nnz"] == two["config"]["nnz_total"]
    peer = mh["modes"]["peer"]
    assert peer["shards"] == 2 and peer["selfcheck_ok"] is True and peer["bcast_B_s"] > 0 and peer["value"] > 0
    assert "skipped" in mh["modes"]["rccl"]                  # RCCL needs distinct devices
    assert two["setup"]["bcast_B_s_modes"]["multi-handle peer"] == peer["bcast_B_s"]
    one = _bench(["--workload", "config2", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-dataset",
                  "--dump-c", str(c1)])
    assert one["n_gpus"] == 1 and one["setup"]["selfcheck_all_ranks_ok"] is True
    a, b = np.load(c2), np.load(c1)
    assert np.array_equal(a["rows"], b["rows"])
    both = a["exact"] & b["exact"]
    assert both.mean() > 0.99
    assert np.array_equal(a["c"][both].view(np.int64), b["c"][both].view(np.int64))
    assert np.isfinite(a["c"]).all()


def test_bench_medium_sample_record():
    r = _bench(["--workload", "medium-sample", "--dataset-stride", "1619", "--dataset-iters", "3",
                "--dataset-warmup", "1", "--dataset-cpu-seconds", "5"])
    assert r["scaling"] == "single-gpu" and r["n_gpus"] == 1 and r["setup"]["selfcheck_failures"] == 0
    assert r["value"] > 0 and r["unit"] == "GFLOP/s"
    rl = r["roofline"]
    assert 0 < rl["p10_frac"] <= rl["median_frac"] <= rl["p90_frac"] < 1.5
    cb = r["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1
    oc = r["oracle_check"]                                   # the CPU leg's oracle C checked this run's C
    assert oc is not None and oc["matrices"] >= 1 and oc["rows_exact"] > 0
    assert oc["exact_rows_not_bitexact"] == 0 and oc["inexact_rows_outside_tol"] == 0


def test_bench_config2_checked_against_cpu_baseline():
    """The headline line on a reduced config-2-shaped matrix: its CPU baseline's C (the oracle on the same A and B)
    checks the GPU's C on every row -- bit-identical rows where the engine reports exact."""
    r = _bench(["--workload", "config2", "--gen", "100000 100000 20 6.6667 normal random 0.05 0 0.5 0.5 14",
                "--steps", "3", "--warmup", "1", "--no-dataset", "--no-multi-handle", "--cpu-warmup", "2",
                "--cpu-seconds", "1"])
    oc = r["cpu_baseline"]["oracle_check"]
    assert oc["ok"] and oc["rows_exact"] == 100000 and oc["exact_mismatch"] == 0
    assert r["setup"]["selfcheck_all_ranks_ok"] is True
