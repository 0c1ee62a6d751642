set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GPMI_LIB_VARIANT=chst timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/chst.log 2>&1 || { tail -20 gpurun_out/chst.log; exit 1; }
grep -m 12 "lds_chol\|loglik" gpurun_out/chst.log
