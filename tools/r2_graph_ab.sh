# GPU tests, then the sparse configs with and without the HIP-graph replay, and
# the dense assembly probe
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not config4 and not config5 and not nu25_n16384" > gpurun_out/r2/pytest_d.log 2>&1 || { tail -30 gpurun_out/r2/pytest_d.log; exit 1; }
tail -3 gpurun_out/r2/pytest_d.log
for g in 0 1; do
  for c in sparse4 sparse5; do
    GPMI_SP_GRAPHS=$g timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r2/gr_${c}_g$g.json 2> gpurun_out/r2/gr_${c}_g$g.err || exit 1
  done
done
timeout -k 10 120 python -u tools/asm_probe.py
