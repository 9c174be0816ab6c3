#!/bin/bash
# Sanity pass on a rebuilt engine: GPU suite, smoke, default bench line (no flags, as the driver runs it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sanity
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sanity/pytest.log 2>&1
rc=$?; tail -n 1 gpurun_out/sanity/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sanity/smoke.log 2>&1
rc=$?; tail -n 1 gpurun_out/sanity/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/sanity/bench.log 2>&1
rc=$?; tail -n 1 gpurun_out/sanity/bench.log | cut -c1-900; exit $rc
