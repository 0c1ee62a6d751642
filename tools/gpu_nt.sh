set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/nt
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 200 python3 tools/lanczos_probe.py sparse5 2>&1 | grep lanczos || exit 1
for cfg in sparse5 sparse4; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 > $D/$cfg.json 2> $D/$cfg.err || { tail -5 $D/$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(d['value'],1), round(d['ms_per_step'],2))"
done
