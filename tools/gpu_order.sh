set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/order
mkdir -p $D
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-band > $D/noband.json 2> $D/noband.err || { tail -5 $D/noband.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/noband.json').read().strip().splitlines()[-1]);print('noband', [(c, round(v['value'],1), round(v['ms_per_step'],2)) for c,v in d['sparse_modes'].items()])"
for cfg in sparse4 sparse5; do
timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 5 > $D/$cfg.json 2> $D/$cfg.err || { tail -5 $D/$cfg.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/$cfg.json').read().strip().splitlines()[-1]);print('$cfg alone', round(d['value'],1), round(d['ms_per_step'],2))"
done
