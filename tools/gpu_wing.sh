# Window SpMM with latency-hidden staging: sparse GPU tests, SpMM timings, then
# sparse5 / sparse4 steps with GPMI_SPMM_WING=1 (default) and 0.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/wing
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for cfg in sparse5 sparse4; do
  for r in 1 0; do
    GPMI_SPMM_WING=$r timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 > $D/$cfg.$r.json 2> $D/$cfg.$r.err || { tail -5 $D/$cfg.$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$cfg.$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$cfg wing=$r', round(d['value'],1), round(d['ms_per_step'],2), r['kernel'], r['avg_launch_ms'], r['frac'])"
  done
done
