#!/usr/bin/env python3
"""tools/sweep_merge.py -- fold the records of resumable sweep calls (gpurun_out/sweep/<name>.*.jsonl) into
profiles/<name>.jsonl.gz (one record per (line, K, dtype); the latest wins) and rewrite profiles/<name>.done, the
dataset indices whose every requested K is present (what tools/sweep_resumable.sh skips next time).

  python tools/sweep_merge.py r03_sweep_medium [--k 1,8,32,128]
"""
import argparse
import gzip
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def read_records(path: Path) -> list[dict]:
    op = gzip.open if path.suffix == ".gz" else open
    out = []
    with op(path, "rt") as f:
        for l in f:
            l = l.strip()
            if l.startswith("{"):
                try:
                    out.append(json.loads(l))
                except ValueError:
                    pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--k", default="1,8,32,128")
    ap.add_argument("--dtype", default="f64")
    args = ap.parse_args()
    ks = {int(x) for x in args.k.split(",")}
    dest = ROOT / "profiles" / f"{args.name}.jsonl.gz"
    recs = {}
    if dest.exists():
        for r in read_records(dest):
            recs[(r["gen"], r["k"], r["dtype"])] = r
    n_old = len(recs)
    for f in sorted((ROOT / "gpurun_out" / "sweep").glob(f"{args.name}.*.jsonl")):
        for r in read_records(f):
            recs[(r["gen"], r["k"], r["dtype"])] = r
    with gzip.open(dest, "wt") as f:
        for key in sorted(recs, key=lambda k: (recs[k].get("idx", -1), k[1], k[2])):
            f.write(json.dumps(recs[key]) + "\n")
    per_idx = {}
    for (g, k, dt), r in recs.items():
        if dt == args.dtype:
            per_idx.setdefault(r["idx"], set()).add(k)
    done = sorted(i for i, s in per_idx.items() if ks <= s)
    (ROOT / "profiles" / f"{args.name}.done").write_text("\n".join(map(str, done)) + "\n")
    shas = sorted({r.get("engine_sha256", "?") for r in recs.values()})
    print(f"{dest.name}: {len(recs)} records ({len(recs) - n_old} new), {len(done)} lines complete; engine builds: "
          + ", ".join(s[:12] for s in shas))


if __name__ == "__main__":
    main()
