#!/usr/bin/env python3
"""tools/pmc_dataset.py -- per-matrix HBM traffic (rocprofv3 PMC) over medium-dataset lines.

BASELINE config 3 asks for "rocprof HBM-BW per matrix".  One driver process (`run`) generates each matrix of the
set (one line ahead on a host thread), plans it at K, and launches `--launches` SpMMs on HBM-resident B and C;
between matrices it launches a one-element torch fill, whose dispatch marks the boundary in the profiler's CSV.
`collect` runs that same driver under rocprofv3 once with --kernel-trace (durations) and once per counter group
(PMC runs never carry other traces; FETCH_SIZE takes 3 of the 4 TCC counters of a pass, so it runs alone, and
WRITE_SIZE (2) shares a pass with TCC_HIT_sum + TCC_MISS_sum), then attributes every engine dispatch
(spmm_rows_kernel / spmm_tile_kernel / spmm_combine_kernel) to its matrix by marker order.

Per matrix and launch (MI355X_MICROARCH.md §HBM): read bytes = 2 x FETCH_SIZE KiB (the gfx950 wide-read correction),
write bytes = WRITE_SIZE KiB; both sit on the L2 memory side, so Infinity-Cache hits are included (L2-miss traffic,
an upper bound on true HBM bytes).  Rate = traffic / kernel time (the union of the engine kernels' intervals: the
matrix-core plans overlap kernels on a side stream).  Each record carries the engine build's
fingerprint (bench.engine_sha256), the L2 requests (TCC_HIT + TCC_MISS) and the gather-ceiling fraction
(bench.achievable); bench.py reads these records for its dataset line.

Sets:  --set stratified --per-class N   N lines of every (avg nnz/row, bw) class, evenly spaced in dataset order
       --set sample --stride S          every S-th dataset line (bench.py's dataset line: S = 80)
  python tools/pmc_dataset.py collect --set sample --stride 160 --out gpurun_out/pmc_dataset/sample160.jsonl
"""
import argparse
import csv
import json
import subprocess
import sys
import time
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
sys.path.insert(0, str(ROOT))
ENGINE = ("spmm_rows_kernel", "spmm_tile_kernel", "spmm_mfma_tile_kernel", "spmm_combine_kernel", "mfma_range_kernel",
          "mfma_fixup_kernel")
PASSES = [["FETCH_SIZE"], ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"]]


def lines_for(args):
    i, n = (int(x) for x in getattr(args, "part", "0/1").split("/"))
    return _lines_for(args)[i::n]


def _lines_for(args):
    from spmm_amd.datasets import medium_dataset_lines
    L = medium_dataset_lines()
    if args.set == "sample":
        return L[args.offset::args.stride]
    cls = defaultdict(list)
    for line in L:
        g = line.split()
        if int(g[0]) * float(g[2]) > args.max_nnz:
            continue
        cls[(int(g[2]), float(g[6]))].append(line)
    out = []
    for key in sorted(cls):
        c = cls[key]
        idx = np.linspace(0, len(c) - 1, args.per_class).round().astype(int)
        out += [c[i] for i in sorted(set(idx))]
    return out


def run(args):
    from concurrent.futures import ThreadPoolExecutor
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    lines = lines_for(args)
    marker = torch.zeros(1, device=dev)
    manifest = []
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    npdt = np.float64 if args.dtype == "f64" else np.float32
    ex = ThreadPoolExecutor(max_workers=1)
    gen = lambda l: S.generate(S.gen_params(l))  # noqa: E731
    fut = ex.submit(gen, lines[0])
    for i, line in enumerate(lines):
        A = fut.result()
        if i + 1 < len(lines):
            fut = ex.submit(gen, lines[i + 1])
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values.astype(npdt), A.m, A.ncols, A.nnz, 0, 0)
        mf.plan(args.k)
        g = torch.Generator(device=dev)
        g.manual_seed(42)
        B = torch.rand((max(A.ncols, 1), args.k), generator=g, device=dev, dtype=tdt)
        Cm = torch.empty((max(A.m, 1), args.k), device=dev, dtype=tdt)
        marker.fill_(1.0)                                   # boundary dispatch
        for _ in range(args.launches):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cm.data_ptr(), args.k, stream.cuda_stream)
        torch.cuda.synchronize()
        inf = mf.info()
        manifest.append({"gen": line, "m": int(A.m), "ncols": int(A.ncols), "nnz": int(A.nnz),
                         "bytes_alg": S.bytes_alg(A.m, A.ncols, A.nnz, args.k, S.F64 if args.dtype == "f64" else S.F32),
                         "tiles": int(inf[19]), "split_rows": int(inf[6]), "windows": int(inf[12])})
        mf.close()
        del B, Cm, A
        print(f"{len(manifest)}/{len(lines)} {line}", flush=True)
    marker.fill_(1.0)
    torch.cuda.synchronize()
    Path(args.manifest).write_text(json.dumps(manifest))


def dispatches(d):
    """[(dispatch id, kernel name, {counter: value})] in dispatch order from a rocprofv3 output directory."""
    rows = defaultdict(lambda: {"name": "", "c": defaultdict(float)})
    files = list(d.rglob("*counter_collection.csv"))
    for f in files:
        for r in csv.DictReader(open(f)):
            e = rows[int(r["Dispatch_Id"])]
            e["name"] = r["Kernel_Name"]
            e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    if not files:
        for f in d.rglob("*kernel_trace.csv"):
            for r in csv.DictReader(open(f)):
                e = rows[int(r["Dispatch_Id"])]
                e["name"] = r["Kernel_Name"]
                e["c"]["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                e["iv"] = (float(r["Start_Timestamp"]), float(r["End_Timestamp"]))
    return [(i, rows[i]["name"], rows[i]["c"], rows[i].get("iv")) for i in sorted(rows)]


def busy_ns(iv):
    """Length of the union of [start, end) intervals: the time at least one engine kernel ran (the matrix-core tiles
    overlap the leftover rows and the exact-range check on a side stream, so summed durations would count twice)."""
    t, end = 0.0, -1e300
    for a, b in sorted(iv):
        if b > end:
            t += b - max(a, end)
            end = b
    return t


def per_matrix(disp, nmat):
    """Split the dispatch list at the marker fills (non-engine kernels between engine runs); sum per matrix."""
    groups, cur, ivs, seen_engine = [], defaultdict(float), [], False
    for _, name, c, iv in disp:
        if any(k in name for k in ENGINE):
            seen_engine = True
            for key, v in c.items():
                cur[key] += v
            if iv:
                ivs.append(iv)
        elif "FillFunctor" in name:                       # the marker (torch fill_), not runtime memsets
            if seen_engine:
                if ivs:
                    cur["busy_ns"] = busy_ns(ivs)
                groups.append(cur)
            cur, ivs, seen_engine = defaultdict(float), [], False
    if len(groups) != nmat:
        raise SystemExit(f"dispatch groups {len(groups)} != matrices {nmat}")
    return groups


def collect(args):
    import bench
    outdir = ROOT / "gpurun_out" / "pmc_dataset" / args.tag
    outdir.mkdir(parents=True, exist_ok=True)
    manifest = outdir / "manifest.json"
    drv = [sys.executable, str(Path(__file__).resolve()), "run", "--set", args.set, "--part", args.part,
           "--per-class", str(args.per_class),
           "--stride", str(args.stride), "--offset", str(args.offset), "--k", str(args.k), "--dtype", args.dtype,
           "--launches", str(args.launches), "--max-nnz", str(args.max_nnz), "--manifest", str(manifest)]
    res = {}
    for i, extra in enumerate([["--kernel-trace"]] + [["--pmc", *p] for p in PASSES]):
        d = outdir / f"pass{i}"
        cmd = ["rocprofv3", *extra, "--output-format", "csv", "-d", str(d), "-o", "p", "--", *drv]
        t0 = time.time()
        with open(outdir / f"pass{i}.log", "w") as log:
            r = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, timeout=args.timeout)
        if r.returncode != 0:
            raise SystemExit(f"pass {i} {extra} failed rc={r.returncode} (see {outdir}/pass{i}.log)")
        man = json.loads(manifest.read_text())
        res[i] = per_matrix(dispatches(d), len(man))
        print(f"pass {i} {extra[-1]}: {len(man)} matrices ({time.time() - t0:.0f}s)", flush=True)
    sha = bench.engine_sha256()
    s = 8 if args.dtype == "f64" else 4
    with open(args.out, "w") as f:
        for j, mrec in enumerate(man):
            L = args.launches
            ms = res[0][j].get("busy_ns", res[0][j]["ns"]) / L / 1e6
            rd = 2.0 * res[1][j]["FETCH_SIZE"] * 1024 / L
            wr = res[2][j]["WRITE_SIZE"] * 1024 / L
            hit, miss = res[2][j].get("TCC_HIT_sum", 0.0) / L, res[2][j].get("TCC_MISS_sum", 0.0) / L
            ach = bench.achievable(ms, rd + wr, hit + miss, float(mrec["ncols"]) * args.k * s, mrec["bytes_alg"])
            rec = {**mrec, "k": args.k, "dtype": args.dtype, "engine_sha256": sha, "kernel_ms": ms,
                   "kernel_sum_ms": res[0][j]["ns"] / L / 1e6,
                   "gflops": 2.0 * mrec["nnz"] * args.k / (ms * 1e-3) / 1e9,
                   "roofline_frac": mrec["bytes_alg"] / (ms * 1e-3) / 8e12,
                   "traffic_bytes": rd + wr, "read_bytes": rd, "write_bytes": wr,
                   "traffic_over_alg": (rd + wr) / mrec["bytes_alg"],
                   "traffic_tbs": (rd + wr) / (ms * 1e-3) / 1e12,
                   "tcc_req": hit + miss, "l2_hit": hit / max(hit + miss, 1.0),
                   "achievable_ms": ach["t_ms"] if ach else None,
                   "frac_of_achievable": ach["frac_of_achievable"] if ach else None,
                   "achievable_bound": ach["bound"] if ach else None}
            f.write(json.dumps(rec) + "\n")
    print(f"wrote {len(man)} records to {args.out}")


def publish(args):
    """Merge collected record files (--inputs) into profiles/pmc_dataset_latest.json, the file bench.py's dataset
    sub-record reads (only records of the current engine build are kept)."""
    import bench
    sha = bench.engine_sha256()
    recs = {}
    for f in args.inputs:
        for l in Path(f).read_text().splitlines():
            if l.startswith("{"):
                r = json.loads(l)
                if r.get("engine_sha256") == sha:
                    recs[(r["gen"], r["k"], r["dtype"])] = r
    dest = ROOT / "profiles" / "pmc_dataset_latest.json"
    dest.write_text(json.dumps({"engine_sha256": sha, "records": list(recs.values())}))
    print(f"{dest}: {len(recs)} records of engine {sha[:12]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "collect", "publish"])
    ap.add_argument("--inputs", nargs="*", default=[])
    ap.add_argument("--set", choices=["stratified", "sample"], default="stratified")
    ap.add_argument("--per-class", type=int, default=6)
    ap.add_argument("--part", default="0/1", help="i/n: every n-th line of the set from i (split a set over calls)")
    ap.add_argument("--stride", type=int, default=160)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--max-nnz", type=float, default=4.0e7)
    ap.add_argument("--timeout", type=int, default=500)
    ap.add_argument("--tag", default="set")
    ap.add_argument("--manifest", default=str(ROOT / "gpurun_out" / "pmc_dataset" / "manifest.json"))
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "pmc_dataset" / "pmc_medium.jsonl"))
    args = ap.parse_args()
    {"run": run, "collect": collect, "publish": publish}[args.mode](args)


if __name__ == "__main__":
    main()
