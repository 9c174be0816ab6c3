#!/bin/bash
# One gpurun session validating the inspector (virtual rows, adaptive block cap, K panels):
# GPU parity tests + smoke, then A/B of inspector policies on config 2 and the medium sweep's weakest matrices.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/insp
mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log; case $rc in 0|1|5) ;; *) exit $rc ;; esac; }
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run tune_cfg2_k32 300 python tools/tune_kernel.py --rounds 3
run tune_cfg2_k128 400 python tools/tune_kernel.py --rounds 3 --k 128
run tune_cfg2_k1 300 python tools/tune_kernel.py --rounds 3 --k 1
run tune_cfg2_k128_f32 400 python tools/tune_kernel.py --rounds 3 --k 128 --dtype f32
run tune_cfg2_k32_f32 300 python tools/tune_kernel.py --rounds 3 --k 32 --dtype f32
run tune_skew_k128 200 python tools/tune_kernel.py --rounds 3 --k 128 --gen "6944 6944 50 16.6667 normal random 0.3 1000 1.4 0.5 14"
run tune_3483_k32 200 python tools/tune_kernel.py --rounds 3 --k 32 --gen "3483 3483 100 33.3333 normal random 0.3 100 0.5 0.95 14"
run tune_698_k8 200 python tools/tune_kernel.py --rounds 3 --k 8 --gen "698 698 500 166.6667 normal random 0.3 0 0.05 0.05 14"
run tune_big_k128 400 python tools/tune_kernel.py --rounds 2 --k 128 --gen "196651 196651 500 166.6667 normal random 0.3 0 0.95 0.05 14"
run bench 600 python bench.py --steps 50 --warmup 10
echo "=== done"
