#!/usr/bin/env python3
"""tools/colperm_probe.py -- does WHERE a block's B rows sit in memory matter?

The four row groups of a wave walk four adjacent rows in step, so on a banded matrix one wave instruction gathers
four B rows with nearby column numbers, i.e. within a few KiB of each other.  This probe relabels the columns by a
permutation p (A' has column p[c] where A has c; B' row p[c] is B row c) and times the engine on (A', B') against
(A, B).  Every row keeps its nonzeros in CSR order, so C' equals C bit for bit (checked); only the addresses of the
gathered B rows change.  Permutations: "random" (adjacent columns land anywhere in B) and "stride" (column c at
position (c * 61) mod n: adjacent columns 61 B rows apart).  Row kernel only (tiles off on both sides), K = 32 fp64.

  python tools/colperm_probe.py --lines "5588 5588 500 166.6667 normal random 0.3 1000 1.9 0.5 14" --k 32
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
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    os.environ["SPMM_HIP_MFMA"] = "-1"
    os.environ["SPMM_HIP_TILES"] = "-1"
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    k = args.k
    for line in args.lines.split(";"):
        A = S.generate(S.gen_params(line))
        n = A.ncols
        rng = np.random.default_rng(7)
        perms = {"identity": np.arange(n, dtype=np.int64), "random": rng.permutation(n),
                 "stride": (np.arange(n, dtype=np.int64) * 61) % n if np.gcd(61, n) == 1 else rng.permutation(n)}
        g = torch.Generator(device=dev)
        g.manual_seed(42)
        B = torch.rand((n, k), generator=g, device=dev, dtype=torch.float64)
        outs = {}
        times = {name: [] for name in perms}
        for _ in range(args.repeat):
            for name, p in perms.items():
                col = p[A.col_idx].astype(np.int32)
                Bp = torch.empty_like(B)
                Bp[torch.from_numpy(p).to(dev)] = B                  # B' row p[c] = B row c
                Cd = torch.empty((A.m, k), device=dev, dtype=torch.float64)
                mf = S.csr_to_format(A.row_ptr, col, A.values, A.m, n, A.nnz, k, 0)
                for _ in range(3):
                    mf.spmm_device(Bp.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, st.cuda_stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.launches):
                    mf.spmm_device(Bp.data_ptr(), S.B_ROW_MAJOR, Cd.data_ptr(), k, st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.launches)
                outs[name] = Cd.cpu().numpy().view(np.int64)
                mf.close()
                del Bp, Cd
        same = {name: bool(np.array_equal(outs[name], outs["identity"])) for name in perms}
        plans = {}
        for name, p in perms.items():
            dp = S.debug_plan(A.row_ptr, p[A.col_idx].astype(np.int32), n, k)
            plans[name] = {f: dp[f] for f in ("xcd", "pair", "lmax", "nwin", "blocks", "fp_lo")}
        best = {name: round(min(v) * 1e3, 2) for name, v in times.items()}
        print(json.dumps({"gen": line, "k": k, "nnz": int(A.nnz), "us": best, "bit_identical": same, "plans": plans,
                          "speedup": {name: round(best["identity"] / best[name], 3) for name in perms}}), flush=True)
        del B


if __name__ == "__main__":
    main()
