# block cyclic reduction: band GPU tests (cyclic reduction ones), then the call timings
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-bcr}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_band.py -m gpu -v -k "cyclic or der" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for m in 0 2; do
  GPMI_BAND_BCR=$m timeout -k 10 120 python -u tools/band_bcr_probe.py > $D/probe_$m.log 2>&1 || { tail -5 $D/probe_$m.log; exit 1; }
  cat $D/probe_$m.log
done
