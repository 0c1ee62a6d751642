set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k batch64 --timeout 200 --timeout-method thread > gpurun_out/t_b64.log 2>&1; rc=$?; tail -25 gpurun_out/t_b64.log; exit $rc
