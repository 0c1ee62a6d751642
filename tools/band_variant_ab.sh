# Dev A/B (round 6): band reductions (N = 16384) with the product library against a timing
# variant (GPMI_LIB_VARIANT=<variant>, built by `make variant`), alternating, 5 refreshes each.
#   bash tools/band_variant_ab.sh <name> <variant>
set -o pipefail
D=gpurun_out/${1:?name}
V=${2:?variant}
mkdir -p $D
for rep in 1 2 3; do
  for v in base $V; do
    if [ $v = base ]; then unset GPMI_LIB_VARIANT; else export GPMI_LIB_VARIANT=$v; fi
    timeout -k 10 200 python -u tools/band_refresh_probe.py 128 5 > $D/band_${v}_$rep.log 2>&1 || { tail -5 $D/band_${v}_$rep.log; exit 1; }
    echo "$v: $(grep refresh $D/band_${v}_$rep.log | awk '{print $4}' | tr '\n' ' ')"
  done
done
