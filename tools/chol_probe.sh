set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/chol_probe.py > gpurun_out/cp_base.log 2>&1


