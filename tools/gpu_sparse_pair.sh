# Column-pair gather SpMM (csr_spmm_pair_kernel): GPU sparse tests, then sparse5 bench
# lines with the pair kernel off (GPMI_SPMM_PAIR=0) and on, and sparse4 with it on.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pair
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
GPMI_SPMM_PAIR=0 timeout -k 10 300 python3 bench.py --config sparse5 --no-cpu-baseline > $O/sparse5_off.json 2> $O/sparse5_off.err || exit 1
timeout -k 10 300 python3 bench.py --config sparse5 --no-cpu-baseline > $O/sparse5_on.json 2> $O/sparse5_on.err || exit 1
timeout -k 10 300 python3 bench.py --config sparse4 --no-cpu-baseline > $O/sparse4_on.json 2> $O/sparse4_on.err || exit 1
for f in sparse5_off sparse5_on sparse4_on; do python3 -c "
import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], r['kernel'], r['avg_launch_ms'], r['frac'])"; done
