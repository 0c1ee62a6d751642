set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s17
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread > gpurun_out/s17/tests.log 2>&1 || { tail -40 gpurun_out/s17/tests.log; exit 1; }
tail -1 gpurun_out/s17/tests.log
for cfg in "GPMI_BAND_QS=0" "GPMI_BAND_QS=1"; do
  echo "== $cfg"; env $cfg timeout -k 10 200 python -u tools/band_probe.py 2>&1 | grep -E "refresh|reduce" || exit 1
done
bash tools/pmc_band.sh && echo pmc ok
