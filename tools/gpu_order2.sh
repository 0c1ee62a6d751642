set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/order2
mkdir -p $D
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/nocpu.json 2> $D/nocpu.err || { tail -5 $D/nocpu.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/nocpu.json').read().strip().splitlines()[-1]);print('band, no cpu', [(c, round(v['value'],1), round(v['ms_per_step'],2)) for c,v in d['sparse_modes'].items()])"
