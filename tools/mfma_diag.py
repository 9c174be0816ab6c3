#!/usr/bin/env python3
"""tools/mfma_diag.py -- one small matrix-core plan, one launch per (K, ring), checked against the oracle: the first
thing to run on a GPU after a change to spmm_mfma.hpp (prints each step before it runs it)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import spmm_amd as S
    from oracle import oracle as O
    line = sys.argv[1] if len(sys.argv) > 1 else "6000 6000 100 33 normal random 0.05 0 0.95 0.95 14"
    A = S.generate(S.gen_params(line))
    dev = torch.device("cuda", 0)
    for k, ring in ((32, "12"), (64, "12"), (32, "6"), (64, "6")):
        os.environ.update(SPMM_HIP_MFMA="1", SPMM_HIP_MFMA_RING=ring)
        print(f"K={k} ring={ring}: plan", flush=True)
        mf = S.csr_to_format(A.row_ptr, A.col_idx, A.values, A.m, A.ncols, A.nnz, k, 0)
        print(f"  tiles {mf.tile_info()}", flush=True)
        x = O.drand48(7 + k, A.ncols * k) * 2.0 - 1.0
        B = torch.from_numpy(np.ascontiguousarray(x.reshape(k, A.ncols).T)).to(dev)
        C = torch.full((A.m, k), float("nan"), dtype=torch.float64, device=dev)
        st = torch.cuda.current_stream(dev)
        print("  launch", flush=True)
        mf.spmm_device(B.data_ptr(), S.B_ROW_MAJOR, C.data_ptr(), k, st.cuda_stream)
        torch.cuda.synchronize()
        print("  synced", flush=True)
        ex = mf.exact_rows()
        y = C.cpu().numpy()
        want = O.spmm(A.row_ptr, A.col_idx, A.values, A.ncols, x, k)
        same = np.array_equal(y[ex].view(np.int64), want[ex].view(np.int64))
        print(f"  exact rows {int(ex.sum())}/{A.m} bit-identical: {same}", flush=True)
        mf.close()


if __name__ == "__main__":
    main()
