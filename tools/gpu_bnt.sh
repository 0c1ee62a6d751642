set -o pipefail
for v in "" bnt0; do echo "variant=$v"; GPMI_LIB_VARIANT=$v timeout -k 10 100 python3 tools/band_refresh_probe.py 128 3 2>&1 | grep -E "refresh" || exit 1; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -1
