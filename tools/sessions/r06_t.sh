#!/bin/bash
# round 6, session t: the shipped engine (08e48ee7) -- config 2 alone under rocprofv3 --kernel-trace --stats (its
# kernel's average duration against the bench line's event time), and the config-5 twins line (fp64 + fp32 vs CPU)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt2 --output-format csv -o kt -- \
    python3 -u bench.py --workload config2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/cfg2_prof.json 2> $OUT/cfg2_prof.err
rc=$?; tail -c 300 $OUT/cfg2_prof.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload twins --steps 10 --warmup 3 > $OUT/twins.json 2> $OUT/twins.err
rc=$?; tail -c 400 $OUT/twins.json; exit $rc
