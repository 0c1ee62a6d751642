# sparse tests + sparse5/sparse4 bench lines (no CPU baseline) + a sparse5 trace
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-sq}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -m gpu -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for cfg in sparse5 sparse4; do
  timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline > $D/bench_$cfg.json 2> $D/bench_$cfg.err || { tail -5 $D/bench_$cfg.err; exit 1; }
done
python - $D <<'PY'
import json, sys
for f in ('bench_sparse5', 'bench_sparse4'):
    d = json.load(open('%s/%s.json' % (sys.argv[1], f)))
    print(f, round(d['value'], 1), 'evals/s', round(d['ms_per_step'], 2), 'ms', 'step frac', d['step_roofline']['frac'], 'spmm frac', d['roofline']['frac'], 'cg it', d['step_roofline']['cg_iterations'])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_sparse5 -o run --output-format csv -- python3 bench.py --config sparse5 --steps 3 --warmup 1 --no-cpu-baseline > $D/bench_prof_sparse5.json 2> $D/bench_prof_sparse5.err
GPMI_MS_MFMA=0 timeout -k 10 200 python -u bench.py --config sparse5 --no-cpu-baseline > $D/bench_sparse5_nomfma.json 2> $D/bench_sparse5_nomfma.err || exit 1
python -c "import json; d=json.load(open('$D/bench_sparse5_nomfma.json')); print('sparse5 GPMI_MS_MFMA=0', round(d['value'],1), round(d['ms_per_step'],2))"
