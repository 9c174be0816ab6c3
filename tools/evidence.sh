#!/bin/bash
# Round-end evidence for the committed engine: GPU suite, smoke, PMC passes (per-launch HBM traffic, written to
# profiles/pmc_latest.json on the box so the bench line below carries it), bench line, rocprofv3 kernel-trace summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?usage: tools/evidence.sh <tag>}
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-400; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pmc 900 python tools/collect_pmc.py --tag $TAG
run bench 600 python bench.py --steps 50 --warmup 10
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "=== done"
