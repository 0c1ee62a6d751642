set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_sparse.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/t_sparse.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/t_sparse.log; tail -1 gpurun_out/t_sparse.log
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bc_$cfg.log 2>&1 || { tail -5 gpurun_out/bc_$cfg.log; exit 1; }
  tail -1 gpurun_out/bc_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$cfg', round(d['value'],1), 'nnz', c['nnz'], 'assembly_s', round(c['assembly_s'],4))"
done
GPMI_SPARSE_BRUTE=1 timeout -k 10 300 python bench.py --config sparse5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bc_brute5.log 2>&1 || exit 1
tail -1 gpurun_out/bc_brute5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('brute sparse5 nnz', c['nnz'], 'assembly_s', round(c['assembly_s'],4))"
