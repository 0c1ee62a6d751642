# Band refresh timings with and without a torch HIP context in the process.
set -o pipefail
export TMPDIR=/tmp
for cfg in "PROBE_TORCH=0" "PROBE_TORCH=1" "PROBE_TORCH=1 GPMI_BAND_LA=0"; do
  echo "== $cfg"; env $cfg timeout -k 10 150 python3 tools/band_refresh_probe.py 128 2 2>&1 | grep refresh || exit 1
done
