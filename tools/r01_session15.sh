#!/bin/bash
# Combine with 8 accumulators + window launch-size rule: GPU suite, affected twins.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s15
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -q
L=$(python -c "import json;d=json.load(open('tools/validation_twins.json'))['twins'];print('\n'.join(d[n] for n in ['rail4284','mawi_201512012345','human_gene1','gupta3','webbase-1M','circuit5M']))")
args=(); while IFS= read -r l; do args+=(--line "$l"); done <<< "$L"
run twins 600 python tools/sweep.py "${args[@]}" --k 32 --dtype f64,f32 --out $OUT/twins_fix.jsonl
echo "=== done"
