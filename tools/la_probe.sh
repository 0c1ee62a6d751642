set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
GPMI_LIB_VARIANT=head timeout -k 10 120 python tools/band_probe.py > gpurun_out/la_head$r.log 2>&1 || exit 1
timeout -k 10 120 python tools/band_probe.py > gpurun_out/la0_$r.log 2>&1 || exit 1
GPMI_BAND_LA=1 GPMI_BAND_LA_GRID=128 timeout -k 10 120 python tools/band_probe.py > gpurun_out/la128_$r.log 2>&1 || exit 1
done
GPMI_BAND_LA=1 GPMI_BAND_LA_GRID=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 200 --timeout-method thread > gpurun_out/la_tests.log 2>&1
