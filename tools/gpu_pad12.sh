set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/pad12
mkdir -p $D
for cfg in sparse4 sparse5; do for pad in 0 2 0 2; do
  GPMI_MSGRAM_PAD=$pad timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 10 > $D/${cfg}_$pad.json 2> $D/${cfg}_$pad.err || { tail -5 $D/${cfg}_$pad.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/${cfg}_$pad.json').read().strip().splitlines()[-1]);print('$cfg pad $pad', round(d['value'],1), round(d['ms_per_step'],2), d['lp_sample'], d['step_roofline']['cg_iterations'])"
done; done
GPMI_MSGRAM_PAD=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --config sparse4 --steps 3 --warmup 1 --no-cpu-baseline > $D/b5.json 2> $D/b5.err
