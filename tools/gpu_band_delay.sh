# Delayed band update: band GPU tests, then reduction timings at N = 16384 for
# GPMI_BAND_DELAY = 1, 2, 4, 8 (nu = 1.5) and the default at nu = 2.5 (panel stats).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-bd}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_band.py -m gpu -v --timeout 400 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for dl in 1 2 4 8; do
  GPMI_BAND_DELAY=$dl timeout -k 10 120 python -u tools/band_refresh_probe.py 128 3 > $D/probe_d$dl.log 2>&1 || { tail -5 $D/probe_d$dl.log; exit 1; }
  echo "delay $dl"; tail -3 $D/probe_d$dl.log
done
timeout -k 10 120 python -u tools/band_refresh_probe.py 128 2 2.5 > $D/probe_nu25.log 2>&1 || exit 1
cat $D/probe_nu25.log
