set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/lznb
mkdir -p $D
for nb in 512 1024 2048 512 1024 2048; do
  GPMI_LZ_NB=$nb timeout -k 10 300 python -u bench.py --config sparse5 --no-cpu-baseline --steps 10 > $D/s5_$nb.json 2> $D/s5_$nb.err || { tail -5 $D/s5_$nb.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/s5_$nb.json').read().strip().splitlines()[-1]);print('nb $nb', round(d['value'],1), round(d['ms_per_step'],2), d['lanczos_orthogonalize']['full_reorth_ms'], d['lp_sample'])"
done
