# Band refresh beside a dense operator that ran a batch of 8 (stream budget check),
# and the dense parity tests.
set -o pipefail
export TMPDIR=/tmp
for cfg in "GPMI_GROUPS=0"; do
  echo "== $cfg"; env $cfg timeout -k 10 200 python -u tools/band_after_dense.py dense-first8 2>&1 | grep -E "cold refresh 1|idle" || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1; tail -1 gpurun_out/parity.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/short_bench.json 2> gpurun_out/short_bench.err || { tail -5 gpurun_out/short_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/short_bench.json').read().strip().splitlines()[-1]);b=d['band_mode'];print(d['value'], d['batch_efficiency'], b['value'], b['reduce_ms'], b['reduction_mfma_frac'])"
