"""Compatibility shim: the dataset recipes live in the package (spmm_amd/datasets.py)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "spmm-research_amd"))
from spmm_amd.datasets import *  # noqa: F401,F403,E402
from spmm_amd.datasets import SHA256_SORTED, medium_dataset_lines, sorted_sha256  # noqa: F401,E402

if __name__ == "__main__":
    L = medium_dataset_lines()
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        print(len(L), sorted_sha256(L) == SHA256_SORTED)
    else:
        sys.stdout.write("\n".join(L) + "\n")
