#!/bin/bash
# round 4 final build, part 1: the GPU suite, smoke, the low-register tile kernel experiment (tools/mfma_lr.hpp),
# config-2 PMC, PMC of the stride-160 dataset sample
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/mfma_probe.py --lr-lib spmm-research_amd/lib/libmfma_probe_lr.so --no-forced --reuse 2 --lines "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14;22354 22354 500 166.6667 normal random 0.6 100 0.95 0.95 14;111476 111476 100 33.3333 normal random 0.3 100 0.95 0.95 14;222214 222214 50 16.6667 normal random 0.05 100 0.95 0.95 14;550072 550072 20 6.6667 normal random 0.6 1000 0.5 0.95 14" > $OUT/probe_lr.log 2>&1; rc=$?; grep -c '^{' $OUT/probe_lr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/collect_pmc.py --tag r04 > $OUT/collect_pmc.log 2>&1; rc=$?; tail -n 2 $OUT/collect_pmc.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/pmc_dataset.py collect --set sample --stride 160 --tag sample160 --out $OUT/pmc_sample160.jsonl > $OUT/pmc_sample160.log 2>&1; rc=$?; tail -n 2 $OUT/pmc_sample160.log; exit $rc
