set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for v in stamps f1oldst; do
GPMI_LIB_VARIANT=$v timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/stamps_$v.log 2>&1 || { tail -20 gpurun_out/stamps_$v.log; exit 1; }
echo "== $v"; grep -m 2 "band_chol" gpurun_out/stamps_$v.log
done
timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/cp.log 2>&1 || exit 1
echo "== new"; cat gpurun_out/cp.log
GPMI_LIB_VARIANT=f1old timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/cp_old.log 2>&1 || exit 1
echo "== f1old"; cat gpurun_out/cp_old.log
