# Band-reduction iteration driver (through gpurun): the band GPU tests, refresh timings
# under look-ahead settings, a probe-build run (GPMI_LIB_VARIANT) and a rocprofv3 kernel
# trace of one refresh without look-ahead (summarise with tools/trace_summary.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${ITER:-it}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in "GPMI_BAND_LA=1" "GPMI_BAND_LA=0" "GPMI_BAND_CQ_LA_GRID=448"; do
  echo "== $cfg"; env $cfg timeout -k 10 100 python3 tools/band_refresh_probe.py 128 2 2>&1 | grep reduce || exit 1
done
if [ -n "$VARIANT" ]; then
  GPMI_LIB_VARIANT=$VARIANT GPMI_BAND_LA=0 timeout -k 10 100 python3 tools/band_refresh_probe.py 128 1 2>&1 | grep -E "cq_recon|reduce" | head -8
fi
GPMI_BAND_LA=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/band_refresh_probe.py 128 1 > $O/probe.log 2>&1
