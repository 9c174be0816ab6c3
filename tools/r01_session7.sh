#!/bin/bash
# Full GPU parity suite + smoke, PMC passes for the bench workload, bench (traffic from the PMC json), rocprof trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s7
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-400; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pmc 700 python tools/collect_pmc.py --tag r01_v5 --steps 5
run bench 600 python bench.py --steps 50 --warmup 10
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "=== done"
