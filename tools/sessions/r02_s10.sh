set -u
mkdir -p gpurun_out/s10
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}"; lscpu | head -20; } > gpurun_out/s10/cpuinfo.txt 2>&1
timeout -k 10 300 python bench.py --workload pipeline --steps 200 --warmup 20 > gpurun_out/s10/pipe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload pipeline --steps 200 --warmup 20 --pipe-m 2048 --pipe-k 512 > gpurun_out/s10/pipe2048.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/s10/bench.log 2>&1 || exit $?
tail -1 gpurun_out/s10/pipe.log; tail -1 gpurun_out/s10/pipe2048.log; tail -1 gpurun_out/s10/bench.log | cut -c1-300
