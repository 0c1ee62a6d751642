set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/spcpu
mkdir -p $D
for cfg in sparse5 sparse4; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 5 > $D/$cfg.json 2> $D/$cfg.err || { tail -5 $D/$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/$cfg.json').read().strip().splitlines()[-1]);cb=d['cpu_baseline'];print('$cfg', round(d['value'],1), round(d['ms_per_step'],2), cb['value'], cb['cg_gram_column_rel_diff_vs_device_max'], cb['slq_logdet_rel_diff_vs_device_same_probes'])"
done
