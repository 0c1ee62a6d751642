set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_band.py -q -k "eigen or traceinv or der" --timeout 120 --timeout-method thread > gpurun_out/t_chase.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/t_chase.log
timeout -k 10 120 python tools/eig_probe.py 128 > gpurun_out/eig_new.log 2>&1 || exit 1
grep -m 3 "eigenvalues\|traceinv\|rel" gpurun_out/eig_new.log
GPMI_CHASE=0 timeout -k 10 120 python tools/eig_probe.py 128 > gpurun_out/eig_old.log 2>&1 || exit 1
grep -m 3 "eigenvalues\|traceinv\|rel" gpurun_out/eig_old.log
