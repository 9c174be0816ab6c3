#!/bin/bash
# VL kernel at 4 waves/SIMD (launch bounds, U/2 strided batch): GPU suite, skewed lines, twins, regression checks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s17
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -q
L=$(python -c "import json;d=json.load(open('tools/validation_twins.json'))['twins'];print('\n'.join(d[n] for n in ['mawi_201512012345','circuit5M','ASIC_680k','rajat30','com-Youtube']))")
args=(); while IFS= read -r l; do args+=(--line "$l"); done <<< "$L"
run twins 600 python tools/sweep.py "${args[@]}" --k 32 --dtype f64,f32 --out $OUT/twins_vl.jsonl
run medskew 600 python tools/sweep.py --line "18448383 18448383 5 1.6667 normal random 0.6 10000 0.05 0.5 14" --line "23478271 23478271 5 1.6667 normal random 0.05 10000 0.05 0.5 14" --line "445906 445906 100 33.3333 normal random 0.6 10000 0.05 0.5 14" --line "2200290 2200290 20 6.6667 normal random 0.05 10000 0.05 0.5 14" --k 1,8,32,128 --out $OUT/medskew.jsonl
run reg 600 python tools/sweep.py --line "1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14" --line "303884 303884 500 166.6667 normal random 0.6 100 1.4 0.95 14" --line "39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14" --k 1,8,32 --out $OUT/reg.jsonl
echo "=== done"
