set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sparse.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/t_sparse.log | tail -30; exit 1; }
tail -1 gpurun_out/t_sparse.log
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || { tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', round(d['value'],1), round(d['ms_per_step'],2), d['lp_sample'])"
done
