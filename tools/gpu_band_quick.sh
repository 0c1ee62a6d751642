# Band quick check: the band GPU tests and refresh timings (default and no look-ahead).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread > gpurun_out/quick/tests.log 2>&1 || { tail -40 gpurun_out/quick/tests.log; exit 1; }
tail -1 gpurun_out/quick/tests.log
for cfg in "GPMI_BAND_LA=1" "GPMI_BAND_LA=0"; do
  echo "== $cfg"; env $cfg timeout -k 10 100 python3 tools/band_refresh_probe.py 128 2 2>&1 | grep refresh || exit 1
done
