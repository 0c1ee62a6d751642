# Band-reduction iteration driver (through gpurun): the band GPU tests, refresh timings
# under look-ahead settings, and a rocprofv3 kernel trace of one refresh without
# look-ahead (summarise with tools/trace_summary.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s12
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread > gpurun_out/s12/tests.log 2>&1 || { tail -40 gpurun_out/s12/tests.log; exit 1; }
tail -2 gpurun_out/s12/tests.log
for cfg in "GPMI_BAND_LA=1" "GPMI_BAND_LA=0" "GPMI_BAND_CQ_LA_GRID=448"; do
  echo "== $cfg"; env $cfg timeout -k 10 100 python3 tools/band_refresh_probe.py 128 2 2>&1 | grep reduce || exit 1
done
GPMI_BAND_LA=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s12/prof -o run -- python3 tools/band_refresh_probe.py 128 1 > gpurun_out/s12/probe.log 2>&1
