set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/p5
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_dense_slq.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for cfg in sparse5 sparse4; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 > $D/$cfg.json 2> $D/$cfg.err || { tail -5 $D/$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(d['value'],1), round(d['ms_per_step'],2))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --config sparse4 --steps 3 --warmup 1 --no-cpu-baseline > $D/b5.json 2> $D/b5.err
