set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/sp4trace -o run --output-format csv -- python3 bench.py --config ${CFG:-sparse4} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sp4trace.log 2>&1 || exit 1
echo ok
