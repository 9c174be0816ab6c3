#!/usr/bin/env python3
"""tools/mfma_engine_trace.py -- launches of the engine on a few lines under named plans (run under rocprofv3
--kernel-trace to split a launch into its kernels, or --pmc for counters): per line, K and plan, --launches launches
(after 3 warm-ups); prints the plan (tile mode, tiles, blocks) and the event-timed ms of each.

  python tools/mfma_engine_trace.py --k 32,128 --plans "np1:SPMM_HIP_MFMA_NP=1;np2:;off:SPMM_HIP_MFMA=-1"
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
LINES = "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;" \
        "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", default=LINES)
    ap.add_argument("--k", default="32")
    ap.add_argument("--plans", default="policy:;off:SPMM_HIP_MFMA=-1")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--repeat", type=int, default=1, help="timed rounds per (line, K, plan), each on a fresh handle")
    ap.add_argument("--plan-fields", default="", help="comma list of spmm_hip_debug_plan fields to record per record "
                    "(host-side plan under the record's environment)")
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    plans = []
    for spec in args.plans.split(";"):
        name, _, kv = spec.partition(":")
        plans.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    for line in args.lines.split(";"):
        A = S.generate(S.gen_params(line))
        for k in (int(x) for x in args.k.split(",")):
            tdt = torch.float64 if args.dtype == "f64" else torch.float32
            vals = A.values if args.dtype == "f64" else A.values.astype("float32")
            B = torch.rand((A.ncols, k), device=dev, dtype=tdt)
            C = torch.empty((A.m, k), device=dev, dtype=tdt)
            for name, env in [p for p in plans for _ in range(args.repeat)]:
                old = {kk: os.environ.get(kk) for kk in env}
                os.environ.update(env)
                mf = S.csr_to_format(A.row_ptr, A.col_idx, vals, A.m, A.ncols, A.nnz, k, 0)
                for _ in range(3):
                    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, st.cuda_stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.launches):
                    mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                for kk, vv in old.items():
                    if vv is None:
                        os.environ.pop(kk, None)
                    else:
                        os.environ[kk] = vv
                inf = mf.info()
                rec = {"gen": line, "k": k, "plan": name, "dtype": args.dtype,
                       "ms": round(e0.elapsed_time(e1) / args.launches, 5),
                       "tile": mf.tile_info(), "info": [int(v) for v in inf]}
                if args.plan_fields:
                    os.environ.update(env)
                    dp = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F64 if args.dtype == "f64" else S.F32)
                    rec["plan_fields"] = {f: dp[f] for f in args.plan_fields.split(",")}
                    for kk, vv in old.items():
                        if vv is None:
                            os.environ.pop(kk, None)
                        else:
                            os.environ[kk] = vv
                print(json.dumps(rec), flush=True)
                mf.close()
            del B, C


if __name__ == "__main__":
    main()
