#!/bin/bash
# round 5 final build, part 1: the GPU suite, smoke, config-2 PMC (profiles/pmc_latest.json), PMC of the stride-160
# dataset sample (published to profiles/pmc_dataset_latest.json on the CPU afterwards)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/collect_pmc.py --tag r05 > $OUT/collect_pmc.log 2>&1; rc=$?; tail -n 2 $OUT/collect_pmc.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/pmc_dataset.py collect --set sample --stride 160 --tag sample160 --out $OUT/pmc_sample160.jsonl > $OUT/pmc_sample160.log 2>&1; rc=$?; tail -n 2 $OUT/pmc_sample160.log; exit $rc
