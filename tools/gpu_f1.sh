set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
GPMI_LIB_VARIANT=chst timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/chst.log 2>&1 || { tail -20 gpurun_out/chst.log; exit 1; }
grep -m 4 "lds_chol" gpurun_out/chst.log
timeout -k 10 120 python tools/chol_probe.py 128 64 > gpurun_out/cp.log 2>&1 || exit 1
cat gpurun_out/cp.log
timeout -k 10 300 python bench.py --no-band --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bd.log 2>&1 || exit 1
tail -1 gpurun_out/bd.log | cut -c1-120
