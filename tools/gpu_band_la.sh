# look-ahead occupancy sweep of the band reduction (N = 16384): SYR2K LDS padding
# (one workgroup per CU) x grid cap
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-la}
mkdir -p $D
run() { GPMI_BAND_LA_LDS=$1 GPMI_BAND_CQ_LA_GRID=$2 timeout -k 10 120 python -u tools/band_refresh_probe.py 128 3 > $D/la_$1_$2.log 2>&1 || exit 1; echo "lds $1 cap $2: $(grep refresh $D/la_$1_$2.log | tr '\n' ' ')"; }
run 0 448
run 8192 224
run 8192 240
run 8192 192
run 8192 160
run 0 384
run 0 320
