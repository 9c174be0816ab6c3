#!/bin/bash
# round 5, session g (verdict r04 item 7): the 8-rank paths rehearsed on one GPU with --dist-backend gloo (ranks share
# cuda:0): config 4 (strong, the 150 M-nonzero gamma line) and the driver's default weak config-2 run; wall time of each
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05g; mkdir -p $OUT
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u bench.py --gpus 8 --workload config4 --scaling strong --dist-backend gloo --steps 5 --warmup 2 \
    --no-cpu-baseline --no-multi-handle > $OUT/config4_8.log 2>&1; rc=$?
echo "config4 x8 ranks: rc=$rc wall $(( $(date +%s) - t0 )) s"; tail -n 1 $OUT/config4_8.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
t0=$(date +%s)
timeout -k 10 900 python -u bench.py --gpus 8 --dist-backend gloo --steps 5 --warmup 2 > $OUT/config2_8.log 2>&1; rc=$?
echo "config2 weak x8 ranks: rc=$rc wall $(( $(date +%s) - t0 )) s"; tail -n 1 $OUT/config2_8.log | cut -c1-300; exit $rc
