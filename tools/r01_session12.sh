#!/bin/bash
# Full GPU suite + medium-sample sweep (v6: windows + vector lanes + XCD order policies).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s12
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -q
run sweep 1000 python tools/sweep.py --dataset medium --stride 160 --k 1,8,32,128 --budget 850 --out $OUT/sweep_medium_s160_v6.jsonl
echo "=== done"
