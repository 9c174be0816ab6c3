set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/mfma/pmc
L="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d gpurun_out/mfma/pmc/p1 -o run --output-format csv -- python3 tools/mfma_probe.py --rmax 32 --reuse 8 --rounds 1 --iters 2 --lines "$L" > gpurun_out/mfma/pmc/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/mfma/pmc/p2 -o run --output-format csv -- python3 tools/mfma_probe.py --rmax 32 --reuse 8 --rounds 1 --iters 2 --lines "$L" > gpurun_out/mfma/pmc/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mfma/pmc/kt -o run --output-format csv -- python3 tools/mfma_probe.py --rmax 32 --reuse 8 --rounds 1 --iters 2 --lines "$L" > gpurun_out/mfma/pmc/kt.log 2>&1
