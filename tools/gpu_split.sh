set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_band.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/t_band.log | tail -20; exit 1; }
tail -1 gpurun_out/t_band.log
timeout -k 10 120 python tools/eig_probe.py 128 > gpurun_out/eig_split.log 2>&1 || exit 1
grep -m 3 "eigenvalues\|rel err" gpurun_out/eig_split.log
GPMI_CHASE_SPLIT=0 timeout -k 10 120 python tools/eig_probe.py 128 > gpurun_out/eig_one.log 2>&1 || exit 1
grep -m 3 "eigenvalues\|rel err" gpurun_out/eig_one.log
