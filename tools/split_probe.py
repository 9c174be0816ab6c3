#!/usr/bin/env python3
"""tools/split_probe.py -- split length T (SPMM_HIP_SEQ_MAX) and vector lanes on small matrices, measured.

For each generator line x K: one handle per setting (the env var is read at plan time), the same HBM-resident B,
launches interleaved over rounds, HIP events; median ms per setting and the engine's plan (T, lanes, split rows).

  python tools/split_probe.py --lines "698 698 500 166.6667 normal random 0.05 0 0.05 0.05 14" --k 32
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", required=True, help="';'-separated generator lines")
    ap.add_argument("--k", default="32")
    ap.add_argument("--settings", default="default;SPMM_HIP_SEQ_MAX=16;SPMM_HIP_SEQ_MAX=32;SPMM_HIP_SEQ_MAX=64;"
                                          "SPMM_HIP_SEQ_MAX=128;SPMM_HIP_SEQ_MAX=256;SPMM_HIP_LANES=64")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    settings = args.settings.split(";")
    for line in args.lines.split(";"):
        A = S.generate(S.gen_params(line))
        for k in (int(x) for x in args.k.split(",")):
            g = torch.Generator(device=dev)
            g.manual_seed(42)
            B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
            hs, outs, res, plans = {}, {}, {}, {}
            for st in settings:
                env = dict(kv.split("=", 1) for kv in st.split(",") if "=" in kv)
                old = {kk: os.environ.get(kk) for kk in env}
                os.environ.update(env)
                mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
                mf.plan(k)
                for kk, vv in old.items():
                    if vv is None:
                        os.environ.pop(kk, None)
                    else:
                        os.environ[kk] = vv
                inf = mf.info()
                plans[st] = {"T": int(inf[8]), "split_rows": int(inf[6]), "lmax": int(inf[16]), "blocks": int(inf[5]),
                             "exact_rows": int(inf[17])}
                hs[st] = mf
                outs[st] = torch.empty((A.m, k), device=dev, dtype=torch.float64)
                res[st] = []
            for _ in range(args.rounds):
                for st, mf in hs.items():
                    run = lambda: mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, outs[st].data_ptr(), k, stream.cuda_stream)  # noqa
                    run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        run()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    res[st].append(e0.elapsed_time(e1) / args.iters)
            ref = outs[settings[0]]
            close = {st: bool(torch.allclose(ref, o, rtol=1e-10, atol=0)) for st, o in outs.items()}
            print(json.dumps({"gen": line, "k": k, "nnz": int(A.nnz),
                              "ms": {st: float(np.median(v)) for st, v in res.items()}, "plan": plans,
                              "close": close}), flush=True)
            for mf in hs.values():
                mf.close()


if __name__ == "__main__":
    main()
