# Dev iteration: syr2k probe, then the named test files (default: all -m gpu).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-iter}
shift
mkdir -p $D
timeout -k 10 200 ./tools/probe/syr2k_probe > $D/syr2k.txt 2>&1 || { echo "probe failed"; tail -5 $D/syr2k.txt; exit 1; }
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
