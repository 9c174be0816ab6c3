#!/bin/bash
# Round-1 measurement session: GPU parity suite, smoke, bench, rocprofv3 kernel stats, PMC traffic, medium sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/s2}
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 50 --warmup 10
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
run pmc 900 python tools/collect_pmc.py --tag ${TAG:-r01_v3}
run sweep 900 python tools/sweep.py --dataset medium --stride 160 --k 1,8,32,128 --budget 600 --out $OUT/sweep_medium_s160_${TAG:-r01_v3}.jsonl
echo "=== done"
