# -m gpu suite + smoke() at the current tree; logs under gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-tests}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
