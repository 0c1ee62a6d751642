set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 300 --timeout-method thread -k "not config5" > gpurun_out/r2/pytest_sp.log 2>&1 || { tail -30 gpurun_out/r2/pytest_sp.log; exit 1; }
tail -2 gpurun_out/r2/pytest_sp.log
for r in 0 1; do
  for c in sparse4 sparse5; do
    GPMI_SPARSE_REORDER=$r timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r2/ro_${c}_r$r.json 2> gpurun_out/r2/ro_${c}_r$r.err || exit 1
  done
done
for c in sparse4 sparse5; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r2/pmc_${c}_fetch -o run --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r2/pmc_${c}_fetch.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r2/pmc_${c}_write -o run --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r2/pmc_${c}_write.log 2>&1 || exit 1
done
