set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_full.log 2>&1 || exit 1
echo prof ok
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_mfma_b64 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band > gpurun_out/pmc_mfma_b64.log 2>&1 || exit 1
echo pmc ok
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-200
done
