set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GPMI_LIB_VARIANT=cstamps timeout -k 10 120 python tools/eig_probe.py 128 > gpurun_out/cstamps.log 2>&1 || { tail -20 gpurun_out/cstamps.log; exit 1; }
grep -m 6 "chase\|eigenvalues" gpurun_out/cstamps.log
