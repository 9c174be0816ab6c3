set -u
mkdir -p gpurun_out/s15
P=$(cat tools/probe_tile_lines.txt)
timeout -k 10 600 python -u tools/ab_tiles.py --lines "$P" --k 32 --dtype f64 --modes=-1,1 --rounds 3 > gpurun_out/s15/probe_k32.jsonl 2> gpurun_out/s15/probe_k32.err || { tail -5 gpurun_out/s15/probe_k32.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/s15/probe_k32.jsonl'):
    d=json.loads(l); print(d['gen'][:52], d['1']['reuse'], d['1']['tiles'], d['1']['speedup'])
"
D="39120 39120 500 166.6667 normal random 0.05 100 0.95 0.95 14"
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  n=$(echo $pmc | cut -c1-12 | tr ' ' _)
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/s15/pmc_$n -o run -- python3 tools/ab_tiles.py --lines "$D" --modes=1 --rounds 1 --iters 2 > gpurun_out/s15/pmc_$n.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s15/prof_pipe -o run -- python3 bench.py --workload pipeline --steps 100 --warmup 10 > gpurun_out/s15/pipe.log 2>&1 || exit $?
tail -1 gpurun_out/s15/pipe.log | cut -c1-300
timeout -k 10 900 python -u bench.py --workload medium-sample --steps 10 --warmup 3 > gpurun_out/s15/medium_sample.log 2>&1 || { tail -5 gpurun_out/s15/medium_sample.log; exit 1; }
tail -1 gpurun_out/s15/medium_sample.log | cut -c1-600
