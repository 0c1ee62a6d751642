# One-pass full-width window SpMM A/B (GPMI_SPMM_FULL=0: the 8-column chunked kernel):
# the sparse GPU tests and the sparse4 / sparse5 bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/spmm
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -q -x --timeout 300 --timeout-method thread > gpurun_out/spmm/tests.log 2>&1 || { tail -30 gpurun_out/spmm/tests.log; exit 1; }
tail -1 gpurun_out/spmm/tests.log
for cfg in sparse4; do
  for full in 1 0; do
    GPMI_SPMM_FULL=$full timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/spmm/b_${cfg}_$full.json 2> gpurun_out/spmm/b_${cfg}_$full.err || { tail -5 gpurun_out/spmm/b_${cfg}_$full.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/spmm/b_${cfg}_$full.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$cfg full=$full', round(d['value'],1), r.get('frac'), r.get('avg_launch_ms', r.get('ms')))"
  done
done
