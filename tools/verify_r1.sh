set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python bench.py --no-band --no-cpu-baseline --eta-per-rank 32 --steps 3 --warmup 1 > gpurun_out/bench_b32.log 2>&1 || exit 1
tail -1 gpurun_out/bench_b32.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
tail -1 gpurun_out/bench_default.log
