#!/bin/bash
# round 6, session v: counters of the row kernel on three low-similarity dense lines and on the same lines with their
# rows sorted by length in groups of 64 (tools/sort_probe.py + tools/sort_pmc.py): one PMC pass each
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06v; mkdir -p $OUT
export TMPDIR=/tmp
i=0
while IFS= read -r L; do
  [ -z "$L" ] && continue
  i=$((i+1)); mkdir -p $OUT/l$i
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_WAIT_INST_ANY TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $OUT/l$i/pa --output-format csv -o pa -- \
      python3 -u tools/sort_probe.py --lines "$L" --k 32 --group 64 --rounds 1 --launches 20 > $OUT/l$i/probe.jsonl 2> $OUT/l$i/probe.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/l$i/probe.err; exit $rc; }
  python -u tools/sort_pmc.py $OUT/l$i --gen "$L" >> $OUT/sort_pmc.jsonl || exit $?
done <<'LINES'
22354 22354 500 166.6667 normal random 0.3 0 0.5 0.05 14
55886 55886 500 166.6667 normal random 0.3 0 0.5 0.05 14
111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14
LINES
wc -l $OUT/sort_pmc.jsonl
