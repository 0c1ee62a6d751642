set -o pipefail
mkdir -p gpurun_out/r2
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print('aff', len(os.sched_getaffinity(0)), 'omp', os.environ.get('OMP_NUM_THREADS'))"; lscpu | head -20) > gpurun_out/r2/host.txt 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r2/bench_dense.json 2> gpurun_out/r2/bench_dense.err && \
timeout -k 10 300 python -u bench.py --config sparse4 > gpurun_out/r2/bench_sparse4.json 2> gpurun_out/r2/bench_sparse4.err && \
timeout -k 10 400 python -u bench.py --config sparse5 > gpurun_out/r2/bench_sparse5.json 2> gpurun_out/r2/bench_sparse5.err
