set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 200 --timeout-method thread -k "eigen" > gpurun_out/eig_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/eig_probe.py > gpurun_out/eig_probe.log 2>&1
