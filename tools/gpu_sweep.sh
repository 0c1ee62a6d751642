set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # label, env..., args
  local label=$1; shift
  timeout -k 10 200 env "$@" > gpurun_out/sw_$label.log 2>&1 || { echo "$label failed"; tail -3 gpurun_out/sw_$label.log; return 1; }
  tail -1 gpurun_out/sw_$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['value'],3), d['roofline']['frac'] if d['roofline'] else None)"
}
B="python3 bench.py --no-band --no-cpu-baseline --steps 2 --warmup 1"
run o16 GPMI_X=0 $B --outer 16 || exit 1
run o8 GPMI_X=0 $B --outer 8 || exit 1
run o24 GPMI_X=0 $B --outer 24 || exit 1
run o32 GPMI_X=0 $B --outer 32 || exit 1
run g2 GPMI_GROUPS=2 $B --outer 16 || exit 1
run sg4 GPMI_SYRK_GROUP=4 $B --outer 16 || exit 1
run sg16 GPMI_SYRK_GROUP=16 $B --outer 16 || exit 1
