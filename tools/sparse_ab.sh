# A/B of an environment knob on the sparse bench lines (no CPU baseline):
#   bash tools/sparse_ab.sh <name> "<ENV=val ...>" [configs...]
set -o pipefail
export TMPDIR=/tmp
NAME=${1:?name}; ENVS=$2; shift 2
D=gpurun_out/$NAME; mkdir -p $D
for cfg in ${@:-sparse4 sparse5}; do
  for v in base alt; do
    if [ $v = alt ]; then E="$ENVS"; else E=""; fi
    env $E timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 10 --warmup 2 --out-json $D/${cfg}_$v.json > $D/${cfg}_$v.log 2>&1 || { tail -20 $D/${cfg}_$v.log; exit 1; }
    python -c "import json; d=json.load(open('$D/${cfg}_$v.json')); print('$cfg $v', round(d['ms_per_step'],3), 'ms', round(d['value'],1), 'evals/s', 'cg_it', d['step_roofline']['cg_iterations'])"
  done
done
