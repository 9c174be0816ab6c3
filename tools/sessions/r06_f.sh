#!/bin/bash
# round 6, session f: would sorting a block's rows by length pay on the texture-bound classes?  (tools/sort_probe.py:
# the shipped engine on each line and on its rows permuted within aligned 16-row groups, K 8 / 32)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/sort_probe.py --lines "$(paste -sd';' tools/r06_sort_lines.txt)" --k 8,32 \
    > $OUT/sort.jsonl 2> $OUT/sort.err
rc=$?; wc -l $OUT/sort.jsonl; exit $rc
