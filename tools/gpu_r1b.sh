set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-band --no-cpu-baseline --eta-per-rank 64 --steps 2 --warmup 1 > gpurun_out/bench_b64.log 2>&1 || exit 1
tail -1 gpurun_out/bench_b64.log | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_b32_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band --eta-per-rank 32 > gpurun_out/pmc_b32_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_b32_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band --eta-per-rank 32 > gpurun_out/pmc_b32_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp4 -o run --output-format csv -- python3 bench.py --config sparse4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sp4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp5 -o run --output-format csv -- python3 bench.py --config sparse5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sp5.log 2>&1 || exit 1
echo done
