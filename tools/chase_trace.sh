set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/chase_prof -o run --output-format csv -- python3 tools/eig_probe.py 64 > gpurun_out/chase_prof.log 2>&1
