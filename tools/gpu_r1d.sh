set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GPMI_LIB_VARIANT=stamps timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
grep -m 6 "band_chol\|loglik" gpurun_out/stamps.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
