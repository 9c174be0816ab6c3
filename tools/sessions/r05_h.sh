#!/bin/bash
# round 5, session h: the GPU suite on the refitted build, the twins line (config 5: fp32 tiles under the fp32 gate,
# verdict r04 item 5), then the small-launch block-capacity A/B (verdict r04 item 6)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload twins --steps 20 --warmup 3 > $OUT/twins.log 2>&1; rc=$?; tail -n 1 $OUT/twins.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/sessions/r05_c.sh
