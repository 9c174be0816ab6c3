#!/bin/bash
# round 6, session s: the row-sort probe (tools/sort_probe.py) on the avg-500 lines that take no tiles at K = 32
# (tools/r06_sort500_lines.txt) -- §6.34 probed avg 20-100 only; a 500-nonzero block is one wave of four rows of
# 500 +- 166 nonzeros, so the wave issues batches for its longest row.  Groups of 16 and 64 rows.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06s; mkdir -p $OUT
export TMPDIR=/tmp
L="$(paste -sd';' tools/r06_sort500_lines.txt)"
timeout -k 10 500 python -u tools/sort_probe.py --lines "$L" --k 32 --group 16 --rounds 2 --launches 10 \
    > $OUT/sort500_g16.jsonl 2> $OUT/sort500_g16.err || exit $?
timeout -k 10 500 python -u tools/sort_probe.py --lines "$L" --k 32 --group 64 --rounds 2 --launches 10 \
    > $OUT/sort500_g64.jsonl 2> $OUT/sort500_g64.err
rc=$?; wc -l $OUT/sort500_g*.jsonl; exit $rc
