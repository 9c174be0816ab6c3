"""bench.py on the GPU (-m gpu): the N>1 path before the driver's 8-GPU run, and the dataset record.

* `bench.py --gpus 2 --dist-backend gloo`: two ranks (self-spawned torch.distributed.run) share cuda:0 -- the
  strong split of config 2 by the reference partitioner (lib/parallel_util.h:141-165), B broadcast, per-rank HIP-event
  timing (value from the slowest rank), C all-gathered once, every rank self-checked.  The gathered C must
  be bit-equal to the one-rank run on every sampled row both runs compute exactly.
  The same run drives the in-process multi-GPU handle of the C ABI (spmm_hip_create_multi, shards on repeated
  device 0): peer B broadcast, spmm_hip_run_sharded timed, C gathered and self-checked.
* `--workload medium-sample` on a small stride: the dataset record's fields (aggregate, fractions, CPU baseline).
* The default line (`--workload dataset`): at N=1 the medium-dataset sample is the value with the config-2 record
  beside it; at N=2 (gloo, one GPU) every rank times its own stride sample and the config-4 strong split (reference
  partitioner, RCCL/gloo B broadcast) rides along -- its gathered C bit-equal to the one-rank run of the same line.
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
    """Run bench.py as a child; its progress (stderr) streams into $SPMM_TEST_LOGDIR/bench_<n>.err when that is set
    (GPU sessions point it under gpurun_out/, so a long record shows progress), else it is captured."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    logdir = os.environ.get("SPMM_TEST_LOGDIR")
    if logdir:
        Path(logdir).mkdir(parents=True, exist_ok=True)
        errp = Path(logdir) / f"bench_{len(list(Path(logdir).glob('bench_*.err')))}.err"
        with open(errp, "w") as ef:
            ef.write(" ".join(args) + "\n")
            ef.flush()
            r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], stdout=subprocess.PIPE, stderr=ef,
                               text=True, env=env, timeout=timeout)
        r.stderr = errp.read_text()
    else:
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
    assert two["setup"]["allgather_C_s"] is not None and "dataset" not in two
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


STRONG_SMALL = "200000 200000 20 6.6667 gamma random 0.3 10000 0.95 0.5 14"   # config 4's shape, 4 M nonzeros


def test_bench_default_line_is_the_dataset_with_config2_beside_it():
    r = _bench(["--dataset-stride", "1619", "--steps", "3", "--warmup", "1", "--dataset-cpu-seconds", "3",
                "--cpu-warmup", "2", "--cpu-seconds", "1"])
    assert r["n_gpus"] == 1 and r["scaling"] == "weak" and r["steps"] == 3 and r["warmup"] == 1
    assert "synthetic_matrices_medium_dataset" in r["config"]["workload"] and r["config"]["matrices"] == 10
    ds = r["dataset"]
    assert ds["iters_per_matrix"] == 3 and ds["warmup_per_matrix"] == 1 and len(ds["ranks"]) == 1
    assert r["ms_per_step"] == pytest.approx(ds["ms_per_pass"], rel=1e-6)
    assert r["value"] == pytest.approx(ds["flops_per_pass"] / (ds["ms_per_pass"] * 1e-3) / 1e9, rel=1e-3)
    rl = r["roofline"]
    assert rl["frac"] == pytest.approx(ds["bytes_alg_per_pass"] / (ds["ms_per_pass"] * 1e-3) / 8e12, rel=2e-3)
    assert r["setup"]["all_ok"] is True and r["setup"]["selfcheck_failures_all_ranks"] == 0
    assert r["oracle_check"]["exact_rows_not_bitexact"] == 0 and r["oracle_check"]["inexact_rows_outside_tol"] == 0
    c2 = r["config2"]                                        # BASELINE configs[1] beside the metric's workload
    assert c2["config"]["nnz_total"] == 19999955 and c2["value"] > 0
    assert c2["cpu_baseline"]["oracle_check"]["ok"] is True
    assert c2["plugin_e2e"] is not None


def test_bench_two_ranks_dataset_and_config4_strong(tmp_path):
    c2, c1 = tmp_path / "strong2.npz", tmp_path / "strong1.npz"
    two = _bench(["--gpus", "2", "--dist-backend", "gloo", "--dataset-stride", "1619", "--steps", "3", "--warmup", "1",
                  "--strong-gen", STRONG_SMALL, "--no-config2", "--dump-c-strong", str(c2)])
    assert two["n_gpus"] == 2 and two["scaling"] == "weak" and two["config"]["dist_backend"] == "gloo"
    ds = two["dataset"]
    assert len(ds["ranks"]) == 2 and all(rr["matrices"] == 10 for rr in ds["ranks"])
    assert two["config"]["matrices"] == 20 and two["setup"]["all_ok"] is True
    assert two["ms_per_step"] == max(rr["ms_per_pass"] for rr in ds["ranks"])
    flops = sum(rr["gflops"] * rr["ms_per_pass"] * 1e-3 * 1e9 for rr in ds["ranks"])
    assert two["value"] == pytest.approx(flops / (two["ms_per_step"] * 1e-3) / 1e9, rel=1e-3)
    st = two["config4_strong"]                                # BASELINE configs[3]: the strong split rides along
    assert st["n_gpus"] == 2 and st["scaling"] == "strong" and st["config"]["workload"].startswith("config4")
    assert sum(st["config"]["nnz_per_rank"]) == st["config"]["nnz_total"]
    assert st["config"]["imbalance_max_over_mean"] >= 1.0
    assert st["roofline"]["kernel_ms_per_launch"] == max(st["roofline"]["kernel_ms_per_rank"]) == st["ms_per_step"]
    assert st["setup"]["selfcheck_all_ranks_ok"] is True and st["setup"]["allgather_C_s"] is not None
    one = _bench(["--workload", "config4", "--gen", STRONG_SMALL, "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                  "--dump-c", str(c1)])
    assert one["config"]["nnz_total"] == st["config"]["nnz_total"]
    a, b = np.load(c2), np.load(c1)
    assert np.array_equal(a["rows"], b["rows"])
    both = a["exact"] & b["exact"]
    assert both.mean() > 0.95
    assert np.array_equal(a["c"][both].view(np.int64), b["c"][both].view(np.int64))
    assert np.isfinite(a["c"]).all()
