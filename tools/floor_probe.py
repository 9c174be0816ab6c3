#!/usr/bin/env python3
"""tools/floor_probe.py -- where the per-call time of SMALL matrices goes (the ~13 us floor of the medium sweep).

For each generator line and K: time `--iters` back-to-back spmm_device calls on one stream with HIP events,
(a) as tools/sweep.py does (the engine records its own timing events around every launch), (b) with
SPMM_HIP_EVENTS=0 (no engine events), (c) the calls captured once into a hipGraph and replayed, and, for scale,
(d) the same count of a 1-element torch kernel.  Run it under `rocprofv3 --kernel-trace --stats` to get the
kernels' own durations.  Prints one JSON line per (line, K).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--line", action="append")
    ap.add_argument("--k", default="1,32")
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    lines = args.line or ["65535 65535 5 1.6667 normal random 0.05 0 0.05 0.05 14",
                          "698 698 500 166.6667 normal random 0.3 0 0.05 0.05 14",
                          "33825 33825 10 3.3333 normal random 0.6 100 0.5 0.95 14",
                          "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"]
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    n = args.iters

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            fn()
            e0.record(stream)
            fn()
            e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n   # us per call

    t = torch.zeros(1, device=dev)
    tiny = timed(lambda: [t.add_(1.0) for _ in range(n)])
    for line in lines:
        A = S.generate(S.gen_params(line))
        for k in [int(x) for x in args.k.split(",")]:
            B = torch.rand((A.ncols, k), device=dev, dtype=torch.float64)
            C = torch.empty((A.m, k), device=dev, dtype=torch.float64)
            rec = {"gen": line, "k": k, "nnz": int(A.nnz), "tiny_torch_us": tiny}
            for mode in ("events", "no_events", "graph"):
                os.environ["SPMM_HIP_EVENTS"] = "0" if mode != "events" else "1"
                mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
                mf.plan(k)
                call = lambda: mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, stream.cuda_stream)  # noqa
                if mode == "graph":
                    with torch.cuda.stream(stream):
                        call()
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=stream):
                        for _ in range(n):
                            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k,
                                           torch.cuda.current_stream().cuda_stream)
                    rec[mode + "_us"] = timed(lambda: g.replay())
                    del g
                else:
                    rec[mode + "_us"] = timed(lambda: [call() for _ in range(n)])
                mf.close()
            os.environ.pop("SPMM_HIP_EVENTS", None)
            print(json.dumps(rec), flush=True)
            del B, C


if __name__ == "__main__":
    main()
