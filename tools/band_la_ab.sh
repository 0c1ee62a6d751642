# Band reduction timings (N = 16384) under GPMI_BAND_LA_FREE values: bash tools/band_la_ab.sh <name> v1 v2 ...
set -o pipefail
export TMPDIR=/tmp
NAME=${1:?name}; shift
D=gpurun_out/$NAME; mkdir -p $D
for v in "$@"; do
  GPMI_BAND_LA_FREE=$v timeout -k 10 200 python -u tools/band_refresh_probe.py 128 3 > $D/la_$v.log 2>&1 || { tail -20 $D/la_$v.log; exit 1; }
  echo "LA_FREE=$v: $(grep refresh $D/la_$v.log | tr '\n' ' ')"
done
