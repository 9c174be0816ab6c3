"""spmm_amd.datasets -- the generator parameter lines of the reference's synthetic datasets (BASELINE configs 2-5).

* ``medium_dataset_lines()`` -- synthetic_matrices_medium_dataset (config 3), restated from its recipe (below).
* ``CONFIG2_LINE`` -- the single headline matrix (config 2).
* ``CONFIG4_LINE`` -- the multi-GPU matrix (config 4): the largest avg-20, skew-10^4 line of
  synthetic_matrices_large_dataset.txt (7,477,550 rows, 150 M nonzeros, 1.8 GB CSR) with ``gamma`` row lengths
  substituted for ``normal`` (the large dataset is all ``normal``; the config asks for gamma/skewed rows).
* ``twins()`` -- the 52 validation twins of config 5 (validation_twins.json: reference config.sh:283-339).

The medium dataset:

Regenerated from the dataset's published recipe (reference matrix_generation_parameters/create_param_file.py:4-68:
three memory ranges 4-32 / 32-512 / 512-2048 MB with 5 sizes each, rows = floor((size*2^20 - 4) / (12*avg + 4)),
std = round(avg/3, 4), normal/random, seed 14) with the grid the published file uses (avg {5,10,20,50,100,500},
bw {0.05,0.3,0.6}, skew {0,100,1000,10000}, neighbours {0.05,0.5,0.95,1.4,1.9}, crs {0.05,0.5,0.95}).  The
published file holds the same lines as a set minus the 10 listed in OMITTED (the tail of the grid); the sorted set's
sha256 is pinned in tests/test_sweep_tools.py.  Only the recipe is restated here -- no data file is copied.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

MEM_RANGES = ["4-32", "32-512", "512-2048"]
PER_RANGE = 5
AVGS = [5, 10, 20, 50, 100, 500]
BWS = [0.05, 0.3, 0.6]
SKEWS = [0, 100, 1000, 10000]
NEIGHS = [0.05, 0.5, 0.95, 1.4, 1.9]
CRSS = [0.05, 0.5, 0.95]
SEED = 14
OMITTED = {
    "303884 303884 500 166.6667 normal random 0.6 10000 1.4 0.95 14",
    "303884 303884 500 166.6667 normal random 0.6 10000 1.9 0.05 14",
    "303884 303884 500 166.6667 normal random 0.6 10000 1.9 0.5 14",
    "303884 303884 500 166.6667 normal random 0.6 10000 1.9 0.95 14",
    "4191 4191 500 166.6667 normal random 0.6 10000 1.9 0.05 14",
    "4191 4191 500 166.6667 normal random 0.6 10000 1.9 0.5 14",
    "4191 4191 500 166.6667 normal random 0.6 10000 1.9 0.95 14",
    "72652 72652 500 166.6667 normal random 0.6 10000 1.9 0.05 14",
    "72652 72652 500 166.6667 normal random 0.6 10000 1.9 0.5 14",
    "72652 72652 500 166.6667 normal random 0.6 10000 1.9 0.95 14",
}
SHA256_SORTED = "c2c07be3a6d28819b294fa13ca62174056d62121d6f36a2922361cc2d39881c0"


def _std(avg: float) -> str:
    v = round(avg / 3, 4)          # numpy.round(avg / 3, 4) in the recipe; same digits for this grid
    return repr(v)


def medium_dataset_lines() -> list[str]:
    out: list[str] = []
    seen: set[str] = set()
    for mr in MEM_RANGES:
        lo, hi = (int(x) for x in mr.split("-"))
        step = int((hi - lo) / PER_RANGE)
        sizes = [i - 1 for i in range(lo + 1, hi, step)][:PER_RANGE]
        for size in sizes:
            for avg in AVGS:
                rows = int((size * (1024 * 1024) - 4) // (12 * avg + 4))
                for bw in BWS:
                    for sk in SKEWS:
                        for ne in NEIGHS:
                            for cr in CRSS:
                                line = " ".join(str(x) for x in
                                                [rows, rows, avg, _std(avg), "normal", "random", bw, sk, ne, cr, SEED])
                                if line not in seen and line not in OMITTED:
                                    seen.add(line)
                                    out.append(line)
    return out


def sorted_sha256(lines: list[str]) -> str:
    return hashlib.sha256("\n".join(sorted(lines)).encode()).hexdigest()


CONFIG2_LINE = "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"
CONFIG4_LINE = "7477550 7477550 20 6.6667 gamma random 0.3 10000 0.95 0.5 14"
CONFIG4_SOURCE = "7477550 7477550 20 6.6667 normal random 0.3 10000 0.95 0.5 14"   # the large-dataset line


def twins() -> dict:
    """validation matrix name -> generator line of its twin (config 5; reference config.sh:283-339)."""
    return json.loads((Path(__file__).resolve().parent / "validation_twins.json").read_text())["twins"]


def stratified_medium(per_class: int = 1, seed: int = 7) -> list[str]:
    """A stratified sample of the medium dataset: ``per_class`` lines of every (avg, bw) class, drawn with a fixed
    seed over sizes, skew, neighbours and similarity (18 classes)."""
    import random
    rng = random.Random(seed)
    by: dict = {}
    for line in medium_dataset_lines():
        f = line.split()
        by.setdefault((float(f[2]), float(f[6])), []).append(line)
    out = []
    for key in sorted(by):
        out.extend(rng.sample(by[key], min(per_class, len(by[key]))))
    return out


if __name__ == "__main__":
    L = medium_dataset_lines()
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        print(len(L), sorted_sha256(L) == SHA256_SORTED)
    else:
        sys.stdout.write("\n".join(L) + "\n")
