set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GPMI_LIB_VARIANT=f1old timeout -k 10 200 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/t_old.log 2>&1; echo "f1old rc=$?"; tail -3 gpurun_out/t_old.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/t_new.log 2>&1; echo "new rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/t_new.log | head -20
