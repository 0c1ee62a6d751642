set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 200 --timeout-method thread > gpurun_out/band_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/band_probe.py > gpurun_out/band_probe.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-der > gpurun_out/bench.log 2>&1
