# A/B of the fused Lanczos (GPMI_LZ_FUSED) on the sparse configs + the GPU tests
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not config4 and not config5 and not nu25_n16384" > gpurun_out/r2/pytest_c.log 2>&1 || { tail -30 gpurun_out/r2/pytest_c.log; exit 1; }
tail -3 gpurun_out/r2/pytest_c.log
for f in 0 1; do
  for c in sparse4 sparse5; do
    GPMI_LZ_FUSED=$f timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r2/ab_${c}_f$f.json 2> gpurun_out/r2/ab_${c}_f$f.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-band > gpurun_out/r2/bench_asm.json 2>gpurun_out/r2/bench_asm.err
