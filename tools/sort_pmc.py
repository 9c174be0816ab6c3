#!/usr/bin/env python3
"""tools/sort_pmc.py -- counters of the row kernel on a line and on the same line with its rows sorted by length
(DESIGN §6.42): does the longest-of-four-rows effect show in the vector-memory instruction count, and does the time
follow it?

Run (one rocprofv3 pass per counter group; each pass runs tools/sort_probe.py's two matrices, --rounds 1):
  rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
      TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d out/pa -o pa --output-format csv \
      -- python3 tools/sort_probe.py --lines "<line>" --k 32 --group 64 --rounds 1 --launches 20
  python tools/sort_pmc.py out --gen "<line>"
The first 23 row-kernel dispatches are the original matrix (3 warm-ups + 20 timed), the next 23 the sorted one.
"""
import argparse
import csv
import glob
import json
from collections import defaultdict
from pathlib import Path


def load(d: Path):
    rows = []
    for f in glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(dict)
    names = {}
    for r in rows:
        if "spmm_rows_kernel" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    ids = sorted(per)
    return [per[i] for i in ids]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--gen", required=True, help="the generator line (its nonzero count normalises the counts)")
    ap.add_argument("--launches", type=int, default=23)
    args = ap.parse_args()
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "spmm-research_amd"))
    import spmm_amd as S
    nnz = float(S.generate(S.gen_params(args.gen)).nnz)
    res = {"orig": {}, "sorted": {}}
    for p in sorted(Path(args.out).iterdir()):
        if not p.is_dir():
            continue
        seq = load(p)
        if len(seq) < 2 * args.launches:
            continue
        for name, part in (("orig", seq[:args.launches]), ("sorted", seq[args.launches:2 * args.launches])):
            for c in part[0]:
                v = sum(d[c] for d in part) / len(part)
                res[name][c] = v
    out = {}
    for name, cs in res.items():
        o = {c: round(v, 1) for c, v in cs.items()}
        for c in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_VALU"):
            if c in cs:
                o[c + "_per_nnz"] = round(cs[c] / nnz, 4)
        out[name] = o
    print(json.dumps({"gen": args.gen, "nnz": nnz, **out}))


if __name__ == "__main__":
    main()
