#!/usr/bin/env python3
"""tools/small_breakdown.py -- where a small launch's time goes (verdict r05 item 5).

Loads the diagnostic build lib/libspmm_hip_stamps.so (make -C spmm-research_amd stamps: the row kernel stores per
block {start, staged, done} in s_memrealtime ticks, 10 ns, one clock for the chip) and, per line and K:
  * event_us      HIP-event time per launch of --launches back-to-back launches (what bench.py reports);
  * single_us     event time of ONE launch on an idle stream (launch + ramp + drain);
  * span_us       first block start -> last block done (the kernel body on the stamps' clock);
  * blocks, blocks/CU and "rounds": how many times the slowest CU's slot was reused (block starts later than the first
                  block's staging);
  * stage_us      median block staging (start -> staged: the prologue's global round trip incl. the barrier);
  * compute_us    median staged -> done (the rows' gather chains and stores); p90 and max (the straggler);
  * tail_us       last block done - p90 of block done times (the grid's drain behind the slowest blocks).
One JSON line per (line, K).  Run the kernel trace beside it (rocprofv3 --kernel-trace) for the launch gaps.

  python tools/small_breakdown.py --lines-file tools/r06_small_lines.txt --k 1,32
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines-file", default=str(ROOT / "tools" / "r06_small_lines.txt"))
    ap.add_argument("--k", default="1,32")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--lib", default=str(ROOT / "spmm-research_amd" / "lib" / "libspmm_hip_stamps.so"))
    args = ap.parse_args()
    import torch
    import spmm_amd as S
    L = S._bind_hip(C.CDLL(args.lib, mode=C.RTLD_LOCAL))
    L.spmm_hip_debug_row_stamps.argtypes = [C.c_void_p]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    lines = [l.strip() for l in open(args.lines_file) if l.strip()]
    for line in lines:
        A = S.generate(S.gen_params(line))
        for k in (int(x) for x in args.k.split(",")):
            h = C.c_void_p()
            assert L.spmm_hip_create(A.row_ptr, A.col_idx, A.values.ctypes.data_as(C.c_void_p), A.m, A.ncols, A.nnz,
                                     k, S.F64, 0, C.byref(h)) == 0
            info = np.zeros(32, np.int64)
            L.spmm_hip_info(h, info)
            nblk = int(info[5])
            g = torch.Generator(device=dev)
            g.manual_seed(42)
            B = torch.rand((A.ncols, k), generator=g, device=dev, dtype=torch.float64)
            Cd = torch.empty((A.m, k), device=dev, dtype=torch.float64)

            def run():
                L.spmm_hip_run_device(h, C.c_void_p(B.data_ptr()), S.B_ROW_MAJOR, C.c_void_p(Cd.data_ptr()), k, sp)
            L.spmm_hip_debug_row_stamps(None)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.launches):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            event_us = e0.elapsed_time(e1) / args.launches * 1e3
            singles = []
            for _ in range(5):
                torch.cuda.synchronize()
                e0.record(st)
                run()
                e1.record(st)
                torch.cuda.synchronize()
                singles.append(e0.elapsed_time(e1) * 1e3)
            stamps = torch.zeros(max(nblk, 1) * 4, dtype=torch.int64, device=dev)
            L.spmm_hip_debug_row_stamps(C.c_void_p(stamps.data_ptr()))
            run()
            torch.cuda.synchronize()
            L.spmm_hip_debug_row_stamps(None)
            s = stamps.cpu().numpy().reshape(-1, 4)[:nblk].astype(np.float64) / 100.0    # ticks -> us
            ok = s[:, 0] > 0
            s = s[ok]
            t0 = s[:, 0].min()
            start, staged, done = s[:, 0] - t0, s[:, 1] - t0, s[:, 2] - t0
            stage = staged - start
            comp = done - staged
            first_staged = np.sort(staged)[0]
            rec = {"gen": line, "k": k, "nnz": int(A.nnz), "m": int(A.m), "blocks": nblk,
                   "blocks_per_cu": round(nblk / 256, 2), "stamped": int(ok.sum()),
                   "event_us": round(event_us, 2), "single_us": round(float(np.median(singles)), 2),
                   "span_us": round(float(done.max()), 2),
                   "late_starts": int((start > first_staged).sum()),
                   "start_spread_us": round(float(np.percentile(start, 90)), 2),
                   "stage_us": round(float(np.median(stage)), 2), "stage_p90_us": round(float(np.percentile(stage, 90)), 2),
                   "compute_us": round(float(np.median(comp)), 2), "compute_p90_us": round(float(np.percentile(comp, 90)), 2),
                   "compute_max_us": round(float(comp.max()), 2),
                   "tail_us": round(float(done.max() - np.percentile(done, 90)), 2),
                   # mean blocks in flight per CU over the span, and the block that ends the launch
                   "active_blocks_per_cu": round(float((done - start).sum() / max(done.max(), 1e-9) / 256), 2),
                   "last_block_start_us": round(float(start[np.argmax(done)]), 2),
                   "last_block_compute_us": round(float(comp[np.argmax(done)]), 2),
                   "max_row_nnz": int(np.diff(A.row_ptr).max()),
                   "tiles": int(info[19]), "split_rows": int(info[6]), "lmax": int(info[16]), "cap": int(info[9]),
                   "seq_max": int(info[8]), "panel_k": int(info[10]), "windows": int(info[12])}
            print(json.dumps(rec), flush=True)
            L.spmm_hip_destroy(h)
            del B, Cd, stamps
        del A


if __name__ == "__main__":
    main()
