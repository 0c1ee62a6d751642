# N=2 rehearsal (two ranks on device 0, gloo) and the look-ahead SYR2K grid cap.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cap
for g in 448 512 384 0; do
  echo "== CQ_LA_GRID=$g"; GPMI_BAND_CQ_LA_GRID=$g timeout -k 10 100 python3 tools/band_refresh_probe.py 128 3 2>&1 | grep -E "refresh" || exit 1
done
bash tools/rehearse_n2.sh > gpurun_out/cap/n2.txt 2>&1 || { tail -20 gpurun_out/n2/dense.log; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/n2/dense.json','gpurun_out/n2/sparse4.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['n_gpus'], d.get('scaling'))"
