# Band reduction timings (N = 16384, three refreshes) under environment settings:
#   bash tools/band_la_ab.sh <name> "<ENV=val ...>" ["<ENV=val ...>" ...]   ("-" = defaults)
set -o pipefail
export TMPDIR=/tmp
NAME=${1:?name}; shift
D=gpurun_out/$NAME; mkdir -p $D
i=0
for E in "$@"; do
  i=$((i + 1))
  [ "$E" = "-" ] && E=""
  env $E timeout -k 10 200 python -u tools/band_refresh_probe.py 128 3 > $D/ab_$i.log 2>&1 || { tail -20 $D/ab_$i.log; exit 1; }
  echo "[$E]: $(grep refresh $D/ab_$i.log | tr '\n' ' ')"
done
