#!/usr/bin/env python3
"""tools/gate_f32_holdout.py -- hold-out lines for the fp32 matrix-core gate (the round-5 fp32 rule was
fitted and chosen on the same 168 lines).

Runs the engine's own gate (spmm_hip_debug_plan, gate-only, fp32) on the host for every --stride-th medium-dataset
line at K 32 and 128 and keeps the (line, K) pairs where the fp32 gate opens and the line is NOT one the round-5 fit
used (tools/r05_fit_lines.txt).  Writes the lines for an on/off A/B on the GPU (tools/mfma_engine_trace.py --dtype
f32 --plans "pol:;off:SPMM_HIP_MFMA=-1").

  python tools/gate_f32_holdout.py --stride 20 --out tools/r06_f32_holdout_lines.txt
"""
import argparse
import json
import sys
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spmm-research_amd"))


def gate(line):
    import spmm_amd as S
    p = S.gen_params(line)
    A = S.generate_masked(p, S.gate_sample_rows(int(p.nr_rows)))
    out = {}
    for k in (32, 128):
        d = S.debug_plan(A.row_ptr, A.col_idx, A.ncols, k, S.F32, 0, gate_only=True)
        out[k] = d["mode"] == "mfma"
    return line, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stride", type=int, default=20)
    ap.add_argument("--offset", type=int, default=7)
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--out", default=str(ROOT / "tools" / "r06_f32_holdout_lines.txt"))
    args = ap.parse_args()
    from spmm_amd.datasets import medium_dataset_lines
    fit = {l.strip() for l in open(ROOT / "tools" / "r05_fit_lines.txt") if l.strip()}
    lines = [l for l in medium_dataset_lines()[args.offset::args.stride] if l not in fit]
    with ProcessPoolExecutor(args.workers) as ex:
        res = list(ex.map(gate, lines, chunksize=4))
    keep = [(l, [k for k, on in o.items() if on]) for l, o in res if any(o.values())]
    Path(args.out).write_text("".join(l + "\n" for l, _ in keep))
    print(json.dumps({"lines_checked": len(lines), "gate_open": len(keep),
                      "k32": sum(32 in ks for _, ks in keep), "k128": sum(128 in ks for _, ks in keep)}))


if __name__ == "__main__":
    main()
