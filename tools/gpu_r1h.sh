set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; echo "main tests rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/tests.log | head -8
GPMI_LIB_VARIANT=nola timeout -k 10 200 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/t_nola.log 2>&1; echo "nola rc=$?"; tail -1 gpurun_out/t_nola.log
GPMI_LIB_VARIANT=stamps timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/stamps.log 2>&1 || exit 1
grep -m 2 "band_chol" gpurun_out/stamps.log
for v in main nola f1old; do
  if [ $v = main ]; then unset GPMI_LIB_VARIANT; else export GPMI_LIB_VARIANT=$v; fi
  timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/cp_$v.log 2>&1 || exit 1
  echo "== $v"; tail -3 gpurun_out/cp_$v.log
done
