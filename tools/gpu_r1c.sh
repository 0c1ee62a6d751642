set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_sparse.log 2>&1 || { tail -30 gpurun_out/tests_sparse.log; exit 1; }
tail -2 gpurun_out/tests_sparse.log
for cfg in sparse4 sparse5; do
  GPMI_SPMM=0 timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${cfg}_v0.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${cfg}_v1.log 2>&1 || exit 1
  for v in v0 v1; do tail -1 gpurun_out/bench_${cfg}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $v', d['value'], d['ms_per_step'], d['roofline'])"; done
done
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_b64_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band > gpurun_out/pmc_b64_fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_b64_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band > gpurun_out/pmc_b64_write.log 2>&1 || exit 1
echo done
