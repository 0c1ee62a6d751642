set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sparse.log 2>&1 || { tail -20 gpurun_out/t_sparse.log; exit 1; }
tail -1 gpurun_out/t_sparse.log
for v in main nont; do
  if [ $v = main ]; then unset GPMI_LIB_VARIANT; else export GPMI_LIB_VARIANT=$v; fi
  for cfg in sparse4 sparse5; do
    timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bnt_${v}_$cfg.log 2>&1 || exit 1
    tail -1 gpurun_out/bnt_${v}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $cfg', round(d['value'],1), d['roofline']['avg_launch_ms'])"
  done
done
unset GPMI_LIB_VARIANT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_sparse5_fetch -o run --output-format csv -- python3 bench.py --config sparse5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_nt.log 2>&1 || exit 1
echo pmc ok
