#!/bin/bash
# Small-matrix floor: engine events vs none vs hipGraph replay, plus rocprof kernel durations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s18
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 12 $OUT/$name.log | cut -c1-400; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run probe 300 python tools/floor_probe.py
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/floor_probe.py --k 1
echo "=== done"
