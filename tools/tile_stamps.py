#!/usr/bin/env python3
"""tools/tile_stamps.py -- where the tile kernel's time goes (measurement only, MI355X).

Plans a matrix with SPMM_HIP_TILES=1 SPMM_HIP_TILE_STAMPS=1, runs a few launches, and reads the per-tile s_memtime
stamps of the last launch: {start, end, cycles parked at the chunk wait + barrier, cycles computing}.  Prints one
JSON line per matrix: launch span, tile duration quantiles, wait and compute shares, start-time spread.
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", required=True)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--env", default="")
    args = ap.parse_args()
    os.environ["SPMM_HIP_TILES"] = "1"
    os.environ["SPMM_HIP_TILE_STAMPS"] = "1"
    for kv in args.env.split(";"):
        if kv:
            k, v = kv.split("=", 1)
            os.environ[k] = v
    import torch
    import spmm_amd as S
    S.hip.spmm_hip_tile_stamps.argtypes = [C.c_void_p, np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS"), C.c_int64]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for line in args.lines.split(";"):
        A = S.generate(S.gen_params(line))
        k = args.k
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
        ti = mf.tile_info()
        B = torch.rand((A.ncols, k), device=dev, dtype=torch.float64)
        Cm = torch.empty((A.m, k), device=dev, dtype=torch.float64)
        for _ in range(5):
            mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cm.data_ptr(), k, stream.cuda_stream)
        torch.cuda.synchronize()
        st = np.zeros(ti["tiles"] * 4, np.int64)
        assert S.hip.spmm_hip_tile_stamps(mf._h, st, len(st)) == 0
        st = st.reshape(-1, 4).astype(np.float64)
        dur = st[:, 1] - st[:, 0]
        t0 = st[:, 0].min()
        q = lambda a, p: float(np.percentile(a, p))
        out = {"gen": line, "tiles": ti["tiles"], "chunks": ti["chunks"], "span": st[:, 1].max() - t0,
               "dur_p10": q(dur, 10), "dur_p50": q(dur, 50), "dur_p90": q(dur, 90), "dur_max": dur.max(),
               "wait_share": float(st[:, 2].sum() / dur.sum()), "comp_share": float(st[:, 3].sum() / dur.sum()),
               "start_p50": q(st[:, 0] - t0, 50), "start_p90": q(st[:, 0] - t0, 90), "start_max": q(st[:, 0] - t0, 100),
               "cyc_per_chunk_wait": float(st[:, 2].sum() / ti["chunks"]),
               "cyc_per_chunk_comp": float(st[:, 3].sum() / ti["chunks"])}
        print(json.dumps(out), flush=True)
        mf.close()


if __name__ == "__main__":
    main()
