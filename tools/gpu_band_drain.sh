# gemm_tile vmcnt drain A/B (GPMI_LIB_VARIANT=nodrain: without) on the band refresh.
set -o pipefail
export TMPDIR=/tmp
for cfg in "GPMI_LIB_VARIANT=nodrain" "X=1" "GPMI_LIB_VARIANT=nodrain" "X=1"; do
  echo "== $cfg"; env $cfg timeout -k 10 100 python3 tools/band_refresh_probe.py 128 2 2>&1 | grep "refresh 1" || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread > gpurun_out/drain_tests.log 2>&1; tail -1 gpurun_out/drain_tests.log
