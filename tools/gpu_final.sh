set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python tools/pcie_probe.py 128 > gpurun_out/pcie.log 2>&1 || { tail -20 gpurun_out/pcie.log; exit 1; }
cat gpurun_out/pcie.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-250
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || { tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-160
done
