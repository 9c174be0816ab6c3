#!/bin/bash
# round 4, session a: matrix-core edge-value tests, instruction chain probe, 64-column waves A/B, bench N=2 (gloo)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/mfma_chain_probe.py --problems 100 > $OUT/chain_probe.jsonl 2> $OUT/chain_probe.err; rc=$?; cat $OUT/chain_probe.jsonl | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -q -k two_ranks --timeout 350 --timeout-method thread > $OUT/pytest_bench.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_bench.log; [ $rc -eq 0 ] || exit $rc
L="39120 39120 500 166.6667 normal random 0.05 0 0.05 0.95 14;39120 39120 500 166.6667 normal random 0.3 0 0.05 0.95 14;22354 22354 500 166.6667 normal random 0.05 0 1.4 0.95 14;196651 196651 500 166.6667 normal random 0.3 0 0.5 0.95 14;111476 111476 100 33.3333 normal random 0.3 0 0.05 0.95 14;445906 445906 100 33.3333 normal random 0.05 0 0.5 0.95 14;222214 222214 50 16.6667 normal random 0.05 0 0.05 0.95 14;550072 550072 20 6.6667 normal random 0.6 0 0.05 0.95 14;4838920 4838920 20 6.6667 normal random 0.05 0 0.5 0.95 14;39120 39120 500 166.6667 normal random 0.05 0 0.05 0.05 14;22354 22354 500 166.6667 normal random 0.05 100 1.4 0.5 14"
timeout -k 10 600 python -u tools/mfma_ab.py --lines "$L" --k 32,64,128 --modes "off:SPMM_HIP_MFMA=-1;np1:SPMM_HIP_MFMA=2,SPMM_HIP_MFMA_NP=1;np2:SPMM_HIP_MFMA=2" --budget 420 > $OUT/ab_np.jsonl 2> $OUT/ab_np.err; rc=$?; wc -l $OUT/ab_np.jsonl; exit $rc
