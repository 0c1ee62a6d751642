set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_band.log 2>&1 || { tail -30 gpurun_out/tests_band.log; exit 1; }
tail -2 gpurun_out/tests_band.log
GPMI_LIB_VARIANT=stamps timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
grep -m 6 "band_chol\|loglik" gpurun_out/stamps.log
timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/cp.log 2>&1 || exit 1
cat gpurun_out/cp.log
