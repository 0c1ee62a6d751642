# Full pass: -m gpu suite + smoke(), then the default bench line (dense + band +
# CPU baselines + sparse_modes). Logs under gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-round}
mkdir -p $D
bash tools/gpu_tests.sh ${1:-round} || exit 1
timeout -k 10 900 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
python - $D <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + '/bench_default.json'))
print('dense', round(d['value'], 2), 'frac', d['roofline']['frac'], 'traffic_src', d['roofline']['traffic_source'])
bm = d['band_mode']
print('band', round(bm['value'], 1), 'reduce', bm['reduce_ms'], 'loglik', bm['loglik_ms'], 'nu25', bm.get('nu25_check'))
print('band batch', {k: v['loglik_ms'] for k, v in bm.get('batch_efficiency', {}).items()})
for k, v in d.get('sparse_modes', {}).items():
    print(k, round(v['value'], 1), 'ms', round(v['ms_per_step'], 2), 'step frac', v['step_roofline']['frac'], 'cpu', v['cpu_baseline']['value'] if v.get('cpu_baseline') else None, 'ref', v.get('reference_check'))
print('cpu dense', d['cpu_baseline']['value'])
PY
