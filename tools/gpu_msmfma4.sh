set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/msmfma4
mkdir -p $D
for v in d m2 m2r0 d m2 m2r0; do
  case $v in d) E="";; m2) E="GPMI_MS_MFMA=2";; m2r0) E="GPMI_MS_MFMA=2 GPMI_MS_RED=0";; esac
  env $E timeout -k 10 300 python -u bench.py --config sparse4 --no-cpu-baseline --steps 20 > $D/s4_$v.json 2> $D/s4_$v.err || { tail -5 $D/s4_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/s4_$v.json').read().strip().splitlines()[-1]);print('$v', round(d['value'],1), round(d['ms_per_step'],2), d['lp_sample'], d['step_roofline']['cg_iterations'])"
done
