#!/bin/bash
# round 6, session b (verdict r05 item 1): the row kernel's access shape on dense-row lines -- tools/shape_probe.py
# (the engine's launch beside gather probes of the same column stream), a kernel trace, and PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06b; mkdir -p $OUT
export TMPDIR=/tmp
L="5588 5588 500 166.6667 normal random 0.3 1000 1.9 0.5 14;111476 111476 100 33.3333 normal random 0.05 0 0.5 0.05 14"
L="$L;22354 22354 500 166.6667 normal random 0.3 100 1.4 0.05 14;4191 4191 500 166.6667 normal random 0.3 0 0.05 0.05 14"
L="$L;1000000 1000000 20 6.6667 normal random 0.3 100 0.95 0.5 14"
timeout -k 10 300 python -u tools/shape_probe.py --lines "$L" > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; cat $OUT/probe.jsonl | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt --output-format csv -o kt -- \
    python3 -u tools/shape_probe.py --lines "$L" --iters 10 > $OUT/kt.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pa --output-format csv -o pa -- \
    python3 -u tools/shape_probe.py --lines "$L" --iters 2 > $OUT/pa.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM \
    SQ_LDS_BANK_CONFLICT TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum \
    TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum \
    -d $OUT/pb --output-format csv -o pb -- python3 -u tools/shape_probe.py --lines "$L" --iters 2 > $OUT/pb.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pc --output-format csv -o pc -- \
    python3 -u tools/shape_probe.py --lines "$L" --iters 2 > $OUT/pc.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pd --output-format csv -o pd -- \
    python3 -u tools/shape_probe.py --lines "$L" --iters 2 > $OUT/pd.log 2>&1
rc=$?; ls $OUT; exit $rc
