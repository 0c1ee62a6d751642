# sparse5 step under SpMM / CG knob variants (no CPU baseline)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-sv}
mkdir -p $D
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --config sparse5 --no-cpu-baseline > $D/$name.json 2> $D/$name.err || { tail -5 $D/$name.err; exit 1; }; python -c "import json; d=json.load(open('$D/$name.json')); print('$name', round(d['value'],1), round(d['ms_per_step'],2), d['roofline']['avg_launch_ms'])"; }
run default GPMI_X=0
run pad_u4 GPMI_MSGRAM_PAD=1 GPMI_SPMM_PUNR=4
run pad_u2 GPMI_MSGRAM_PAD=1 GPMI_SPMM_PUNR=2
run u4 GPMI_SPMM_PUNR=4
