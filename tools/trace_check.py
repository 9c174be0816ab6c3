#!/usr/bin/env python3
"""tools/trace_check.py -- the bench line's dataset time against the profiler's kernel trace of the same run.

bench.py times each matrix's --steps launches with HIP events behind a GPU spin kernel (the pre-roll).  Under
`rocprofv3 --kernel-trace` that spin kernel marks the start of each timed batch, so the engine dispatches between a
spin kernel and the next non-engine dispatch are exactly one matrix's timed launches.  Their busy time (the union of
the dispatch intervals: matrix-core plans overlap kernels on a side stream) / steps is the profiler's kernel time per
launch; this tool pairs it, in order, with the per-matrix records of `bench.py --dataset-out` and prints the sums,
the per-matrix ratio spread and the roofline fraction recomputed from the trace.

  rocprofv3 --kernel-trace --stats -d out -o kt -- python3 bench.py --steps 20 --warmup 5 --dataset-out ds.jsonl
  python tools/trace_check.py out/.../kt_kernel_trace.csv ds.jsonl --steps 20
"""
import argparse
import csv
import json

import numpy as np

ENGINE = ("spmm_rows_kernel", "spmm_ring_kernel", "spmm_tile_kernel", "spmm_mfma_tile_kernel", "spmm_combine_kernel", "mfma_range_kernel",
          "mfma_fixup_kernel")


def busy(iv):
    t, end = 0.0, -1e300
    for a, b in sorted(iv):
        if b > end:
            t += b - max(a, end)
            end = b
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("dataset")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    recs = [json.loads(l) for l in open(args.dataset)]
    batches, cur, open_ = [], [], False
    for r in rows:
        name = r["Kernel_Name"]
        if "spin_kernel" in name:
            if open_ and cur:
                batches.append(cur)
            cur, open_ = [], True
            continue
        if any(k in name for k in ENGINE):
            if open_:
                cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        elif open_:
            if cur:
                batches.append(cur)
            cur, open_ = [], False
    if open_ and cur:
        batches.append(cur)
    # the dataset's batches are the last len(recs) ones (config 2's timed batch comes first)
    batches = batches[-len(recs):]
    assert len(batches) == len(recs), (len(batches), len(recs))
    tr = np.array([busy(b) / args.steps / 1e6 for b in batches])          # ms per launch
    ev = np.array([r["ms"] for r in recs])
    by = np.array([r["bytes_alg"] for r in recs])
    fl = np.array([r["flops"] for r in recs])
    ratio = tr / ev
    out = {"matrices": len(recs), "event_ms_per_pass": round(float(ev.sum()), 4),
           "trace_busy_ms_per_pass": round(float(tr.sum()), 4), "trace_over_event": round(float(tr.sum() / ev.sum()), 4),
           "per_matrix_trace_over_event": {"p10": round(float(np.percentile(ratio, 10)), 4),
                                           "median": round(float(np.median(ratio)), 4),
                                           "p90": round(float(np.percentile(ratio, 90)), 4)},
           "gflops_event": round(float(fl.sum() / ev.sum() / 1e6), 2),
           "gflops_trace": round(float(fl.sum() / tr.sum() / 1e6), 2),
           "roofline_frac_event": round(float(by.sum() / ev.sum() / 1e6 / 8000.0), 4),
           "roofline_frac_trace": round(float(by.sum() / tr.sum() / 1e6 / 8000.0), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
