#!/usr/bin/env python3
"""tools/mfma_engine_trace.py -- launches of the engine's default plan on a few lines (run under rocprofv3
--kernel-trace to split the launch into its kernels): per line, 20 launches with the policy plan, then 20 with
matrix-core tiles off; prints the plan (tile mode, tiles, blocks) and the event-timed ms of each."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
LINES = ["39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14",
         "111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14"]


def main():
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    k = 32
    for line in LINES:
        A = S.generate(S.gen_params(line))
        B = torch.rand((A.ncols, k), device=dev, dtype=torch.float64)
        C = torch.empty((A.m, k), device=dev, dtype=torch.float64)
        for name, env in (("policy", {}), ("off", {"SPMM_HIP_MFMA": "-1"})):
            os.environ.update(env)
            mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
            for kk in env:
                os.environ.pop(kk)
            for _ in range(3):
                mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            inf = mf.info()
            print(json.dumps({"gen": line, "plan": name, "ms": round(e0.elapsed_time(e1) / 20, 5),
                              "tile": mf.tile_info(), "info": [int(v) for v in inf]}), flush=True)
            mf.close()


if __name__ == "__main__":
    main()
