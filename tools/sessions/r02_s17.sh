set -u
mkdir -p gpurun_out/pmc_dataset
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/pmc_dataset.py collect --per-class 16 --k 32 --max-nnz 6e7 --timeout 600 --out gpurun_out/pmc_dataset/r02_pmc_medium_k32.jsonl > gpurun_out/pmc_dataset/collect.log 2>&1 || { tail -20 gpurun_out/pmc_dataset/collect.log; tail -20 gpurun_out/pmc_dataset/pass*.log | tail -40; exit 1; }
tail -5 gpurun_out/pmc_dataset/collect.log
