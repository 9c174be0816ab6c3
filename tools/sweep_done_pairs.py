#!/usr/bin/env python3
"""tools/sweep_done_pairs.py -- the (line, K) pairs already measured by tools/sweep.py record files, as 'K<TAB>line'
(sweep.py --skip-pairs), so a sweep split over several GPU calls resumes where the last call stopped.

  python tools/sweep_done_pairs.py gpurun_out/sweep/r04_ab_changed.*.jsonl --out profiles/r04/ab_done_pairs.txt
"""
import argparse
import glob
import json
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    done = set()
    for pat in args.files:
        for f in glob.glob(pat):
            for l in open(f):
                if l.startswith("{"):
                    d = json.loads(l)
                    if "ms_base" in d:
                        done.add(f"{d['k']}\t{d['gen']}")
    Path(args.out).write_text("".join(x + "\n" for x in sorted(done)))
    print(f"{args.out}: {len(done)} pairs")


if __name__ == "__main__":
    main()
