# sparse4 with the one-pass window SpMM: GPU sparse tests, PMC FETCH / WRITE passes of
# bench.py --config sparse4 (summarise with PMC_LAST=50 tools/pmc_summary.py), bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sp4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --config sparse4 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py --config sparse4 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit 1
echo pmc ok
