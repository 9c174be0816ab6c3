#!/usr/bin/env python3
"""tools/sweep_flag.py -- (line, K) pairs of a sweep whose timing is suspect, as a 'K<TAB>generator line' file for
`tools/sweep.py --pairs` (re-timed in a later call; tools/sweep_merge.py keeps the latest record).

A record is flagged when
  * its timed batches disagree (slowest / fastest batch > --batch-spread): something else used the GPU during it, or
  * the reference sweep (--ref, e.g. the round-3 config-3 records) ran the SAME plan (no tiles in either, same
    blocks, K panel, windows and split rows) more than --ref-ratio times faster.
Round 5: another worker's allocations, uploads and frees stretched K = 128 timed regions of lines over 10 M nonzeros
by up to 2x in two sweep calls (52 % and 17 % of those records, 3 % in the third); the first rule alone misses a
region that is slow from its first batch to its last.

  python tools/sweep_flag.py profiles/r05_sweep_medium.jsonl.gz --ref profiles/r03_sweep_medium.jsonl.gz \\
      --out tools/r05_retime_pairs.txt
"""
import argparse
import gzip
import json
from collections import Counter


def load(path):
    op = gzip.open if path.endswith(".gz") else open
    out = {}
    with op(path, "rt") as f:
        for l in f:
            if l.startswith("{"):
                r = json.loads(l)
                if r.get("dtype", "f64") == "f64":
                    out[(r["gen"], int(r["k"]))] = r
    return out


PLAN = ("blocks", "panel_k", "windows", "split_rows")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sweep")
    ap.add_argument("--ref", default=None)
    ap.add_argument("--batch-spread", type=float, default=1.25)
    ap.add_argument("--ref-ratio", type=float, default=1.3)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    new = load(args.sweep)
    ref = load(args.ref) if args.ref else {}
    flagged, why = [], Counter()
    for key, r in new.items():
        b = r.get("batches") or []
        spread = max(b) / min(b) if len(b) > 1 and min(b) > 0 else 1.0
        o = ref.get(key)
        same_plan = (o is not None and r.get("tiles", 0) == 0 and o.get("tiles", 0) == 0
                     and all(r.get(f) == o.get(f) for f in PLAN))
        if spread > args.batch_spread:
            flagged.append(key)
            why["batch spread"] += 1
        elif same_plan and r["ms"] > args.ref_ratio * o["ms"]:
            flagged.append(key)
            why["slower than the same plan in --ref"] += 1
    with open(args.out, "w") as f:
        for g, k in sorted(flagged, key=lambda x: (x[1], x[0])):
            f.write(f"{k}\t{g}\n")
    byk = Counter(k for _, k in flagged)
    print(f"{len(flagged)} of {len(new)} records flagged ({dict(why)}); per K {dict(sorted(byk.items()))}; "
          f"{len({g for g, _ in flagged})} lines -> {args.out}")


if __name__ == "__main__":
    main()
