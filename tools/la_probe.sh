set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 120 python tools/band_probe.py > gpurun_out/ab_1024_$r.log 2>&1 || exit 1
GPMI_LIB_VARIANT=d2048 timeout -k 10 120 python tools/band_probe.py > gpurun_out/ab_2048_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 200 --timeout-method thread > gpurun_out/la_tests.log 2>&1
