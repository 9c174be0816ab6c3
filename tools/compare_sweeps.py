#!/usr/bin/env python3
"""tools/compare_sweeps.py OLD.jsonl NEW.jsonl -- per-K geometric-mean speedup, parity, worst regressions."""
import json
import sys

import numpy as np


def load(p):
    return {(d["gen"], d["k"], d.get("dtype", "f64")): d for d in map(json.loads, open(p))}


def main():
    old, new = load(sys.argv[1]), load(sys.argv[2])
    common = [k for k in new if k in old]
    r = np.array([old[k]["ms"] / new[k]["ms"] for k in common])
    print(f"{len(new)} new records, {len(common)} in common; speedup geo-mean {np.exp(np.log(r).mean()):.3f} "
          f"min {r.min():.3f} max {r.max():.3f}")
    for K in sorted({k[1] for k in common}):
        rr = np.array([old[k]["ms"] / new[k]["ms"] for k in common if k[1] == K])
        print(f"  K={K:4d}: geo {np.exp(np.log(rr).mean()):.3f} min {rr.min():.3f} max {rr.max():.3f}")
    bad = [k for k in new if not (new[k]["bitexact_seq_rows"] and new[k]["normwise_ok"])]
    print("parity failures:", len(bad), bad[:3])
    print("worst regressions:")
    for k in sorted(common, key=lambda k: old[k]["ms"] / new[k]["ms"])[:int(sys.argv[3]) if len(sys.argv) > 3 else 8]:
        d = new[k]
        print(f"  {k[0]!r} K={k[1]}: {old[k]['ms']:.4f} -> {d['ms']:.4f} ms  T={d.get('seq_max')} "
              f"split={d.get('split_rows')} panel_k={d.get('panel_k')}")


if __name__ == "__main__":
    main()
