# Round-end GPU pass: -m gpu suite, smoke(), default bench (dense + band + CPU
# baseline), the sparse configs, and a rocprofv3 kernel-trace of the default
# bench (its stats are copied to profiles/).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || { tail -30 gpurun_out/final/tests.log; exit 1; }
tail -1 gpurun_out/final/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail -5 gpurun_out/final/bench_default.err; exit 1; }
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python -u bench.py --config $cfg > gpurun_out/final/bench_$cfg.json 2> gpurun_out/final/bench_$cfg.err || { tail -5 gpurun_out/final/bench_$cfg.err; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/final/bench_under_rocprof.json 2> gpurun_out/final/bench_under_rocprof.err
