#!/bin/bash
# round 6, session y: the final engine (paired short rows + wide window)'s PMC records -- config 2 (profiles/pmc_latest.json, the config-2 record's
# traffic) and every 80th medium-dataset line at K = 32 (the bench line's per-matrix traffic and gather ceiling).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/collect_pmc.py --tag r06 --steps 5 > $OUT/collect_pmc.log 2>&1
rc=$?; tail -n 3 $OUT/collect_pmc.log; [ $rc -eq 0 ] || exit $rc
for P in 0 1; do
  timeout -k 10 1000 python -u tools/pmc_dataset.py collect --set sample --stride 80 --part $P/2 --k 32 \
      --timeout 450 --tag s80_p$P --out $OUT/pmc_s80_p$P.jsonl > $OUT/pmc_s80_p$P.log 2>&1
  rc=$?; tail -n 2 $OUT/pmc_s80_p$P.log; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_dataset.py publish --inputs $OUT/pmc_s80_p0.jsonl $OUT/pmc_s80_p1.jsonl
cp profiles/pmc_dataset_latest.json profiles/pmc_r06.json profiles/pmc_latest.json $OUT/
exit 0
