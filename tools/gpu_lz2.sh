set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/lz2
mkdir -p $D
for nr in 512 1024 2048 256; do echo "LZ_NB=$nr"; GPMI_LZ_NB=$nr timeout -k 10 200 python3 tools/lanczos_probe.py sparse5 2>&1 | grep lanczos || exit 1; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_dense_slq.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python -u bench.py --config sparse5 --no-cpu-baseline > $D/b5.json 2> $D/b5.err || { tail -5 $D/b5.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/b5.json').read().strip().splitlines()[-1]);print('sparse5', round(d['value'],1), round(d['ms_per_step'],2))"
