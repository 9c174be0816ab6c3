#!/bin/bash
# round 6, session r: column relabeling probe (tools/colperm_probe.py) -- the same matrices with their
# columns (and B's rows) permuted, row kernel only, K = 32 fp64: does the address spread of a wave's four gathers matter?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06r; mkdir -p $OUT
export TMPDIR=/tmp
L="5588 5588 500 166.6667 normal random 0.3 1000 1.9 0.5 14;4191 4191 500 166.6667 normal random 0.3 0 0.05 0.05 14"
L="$L;22354 22354 500 166.6667 normal random 0.3 0 0.5 0.05 14;5588 5588 500 166.6667 normal random 0.05 100 0.95 0.95 14"
L="$L;111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14;20901 20901 100 33.3333 normal random 0.05 0 0.05 0.05 14"
L="$L;362298 362298 100 33.3333 normal random 0.6 0 0.5 0.05 14;1082401 1082401 10 3.3333 normal random 0.3 0 0.5 0.05 14"
L="$L;2097151 2097151 5 1.6667 normal random 0.05 0 0.5 0.05 14;1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"
timeout -k 10 900 python -u tools/colperm_probe.py --lines "$L" --k 32 > $OUT/colperm.jsonl 2> $OUT/colperm.err
rc=$?; wc -l $OUT/colperm.jsonl; exit $rc
