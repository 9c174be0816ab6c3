"""Sweep tooling (CPU): the medium dataset regenerated from its recipe equals the published file (pinned hash)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))


def test_medium_dataset_lines_match_published_set():
    from spmm_amd.datasets import medium_dataset_lines, sorted_sha256, SHA256_SORTED
    L = medium_dataset_lines()
    assert len(L) == 16190 and len(set(L)) == 16190
    assert sorted_sha256(L) == SHA256_SORTED
    for line in L[:50] + L[-50:]:
        f = line.split()
        assert len(f) == 11 and f[4] == "normal" and f[5] == "random" and f[10] == "14"
