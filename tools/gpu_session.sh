#!/bin/bash
# tools/gpu_session.sh -- one gpurun session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault / abort / segfault / timeout ends the session (no retries).
# Ordinary test failures (pytest exit 1) do not stop the later measurement steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    case $rc in
        0|1|5) return 0 ;;             # ok / test failures / no tests collected
        *) echo "STOP: $name ended with $rc"; exit $rc ;;
    esac
}
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == tests ]]; then
    step pytest_gpu 1500 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
    step bench 600 python bench.py --steps 50 --warmup 10
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
fi
echo "=== done"
