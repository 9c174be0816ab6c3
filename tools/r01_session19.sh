#!/bin/bash
# Fused split-row combine + events off by default + int4 block table: GPU suite, floor probe, bench, small sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s19
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 12 $OUT/$name.log | cut -c1-400; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run fused 600 python -u -m pytest tests/test_gpu_fused_combine.py -x -v --timeout 120 --timeout-method thread
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run probe 300 python tools/floor_probe.py
run bench 600 python bench.py --steps 50 --warmup 10
run sweep 900 python tools/sweep.py --stride 160 --k 1,8,32,128 --out $OUT/sweep_s160_v7.jsonl
echo "=== done"
