# Short bench (no CPU baseline) + the forced whole-reduction fallback test.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/short
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -q -x --timeout 200 --timeout-method thread -k "redoes_reduction" > gpurun_out/short/tests.log 2>&1 || { tail -30 gpurun_out/short/tests.log; exit 1; }
tail -1 gpurun_out/short/tests.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/short/bench.json 2> gpurun_out/short/bench.err || { tail -5 gpurun_out/short/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/short/bench.json').read().strip().splitlines()[-1]);b=d['band_mode'];print(d['value'], b['value'], b['reduce_ms'], b['reduction_mfma_frac'], b['panel'])"
