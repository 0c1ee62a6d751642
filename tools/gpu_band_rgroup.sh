# Look-ahead SYR2K tile order: band GPU tests at the default, then refresh timings
# per GPMI_BAND_RGROUP (0: plain triangle order).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-rgroup}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for g in 0 4 8 16 32; do
  echo "== RGROUP=$g"; GPMI_BAND_RGROUP=$g timeout -k 10 100 python3 tools/band_refresh_probe.py 128 3 2>&1 | grep -E "refresh|first" || exit 1
done
