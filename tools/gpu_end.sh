set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_final.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_full.log 2>&1 || exit 1
echo prof ok
