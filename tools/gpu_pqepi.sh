set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/pqepi
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_dense_slq.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for cfg in sparse5 sparse4; do
  for r in 1 0; do
    GPMI_MS_PQEPI=$r timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 > $D/$cfg.$r.json 2> $D/$cfg.$r.err || { tail -5 $D/$cfg.$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$D/$cfg.$r.json').read().strip().splitlines()[-1]);print('$cfg pqepi=$r', round(d['value'],1), round(d['ms_per_step'],2), d['reference_check'].get('gram_rel_err'))"
  done
done
