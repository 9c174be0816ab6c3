#!/usr/bin/env python3
"""tools/sort_probe.py -- would sorting a block's rows by length pay?  (round 6)

The shape probe (§6.31) found the avg-100 lines bound by the texture unit, which pays for the LONGEST of the four
rows a wave walks in step (vector-memory instructions 1.34x the mean-row count).  Before changing the kernel, this
measures the effect with the shipped engine: each line's rows are permuted within aligned groups of --group rows
(sorted by length, longest first), so a wave's four row groups get rows of similar length, and the unmodified engine
runs both the original and the permuted matrix (same B, HIP events, interleaved rounds).  The cost shows too: the
four rows of a wave are no longer consecutive, so similar rows lose the in-step merge of their common columns.

  python tools/sort_probe.py --lines "111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14;..." --k 32
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def permuted(S, A, group):
    lens = np.diff(A.row_ptr)
    m = A.m
    perm = np.arange(m)
    for s in range(0, m, group):
        e = min(m, s + group)
        perm[s:e] = s + np.argsort(-lens[s:e], kind="stable")
    newlens = lens[perm]
    rp = np.concatenate([[0], np.cumsum(newlens)]).astype(np.int32)
    idx = np.concatenate([np.arange(A.row_ptr[r], A.row_ptr[r + 1]) for r in perm]) if A.nnz else np.zeros(0, int)
    return S.CSR(rp, A.col_idx[idx].copy(), A.values[idx].copy(), m, A.ncols), perm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", required=True)
    ap.add_argument("--k", default="32")
    ap.add_argument("--group", type=int, default=16)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for line in [x.strip() for x in args.lines.split(";") if x.strip()]:
        A = S.generate(S.gen_params(line))
        P, perm = permuted(S, A, args.group)
        for k in (int(x) for x in args.k.split(",")):
            g = torch.Generator(device=dev)
            g.manual_seed(42)
            B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
            hs = {n: S.csr_to_format(M.row_ptr, M.col_idx, M.values, M.m, M.ncols, M.nnz, k, 0) for n, M in
                  (("orig", A), ("sorted", P))}
            Cs = {n: torch.empty((A.m, k), device=dev, dtype=torch.float64) for n in hs}
            ms = {n: [] for n in hs}
            for _ in range(args.rounds):
                for n, mf in hs.items():
                    run = lambda: mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, Cs[n].data_ptr(), k, st.cuda_stream)  # noqa
                    for _ in range(3):
                        run()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(args.launches):
                        run()
                    e1.record(st)
                    torch.cuda.synchronize()
                    ms[n].append(e0.elapsed_time(e1) / args.launches)
            same = bool(torch.equal(Cs["orig"][torch.from_numpy(perm).to(dev)], Cs["sorted"]))
            info = {n: [int(v) for v in mf.info()[[5, 6, 16, 19]]] for n, mf in hs.items()}
            for mf in hs.values():
                mf.close()
            o, s_ = min(ms["orig"]), min(ms["sorted"])
            print(json.dumps({"gen": line, "k": k, "ms_orig": round(o, 5), "ms_sorted": round(s_, 5),
                              "speedup": round(o / s_, 4), "same_bits": same, "blocks_split_lmax_tiles": info}),
                  flush=True)
            del B, Cs


if __name__ == "__main__":
    main()
