# Summaries of a tools/gpu.sh run's traces and PMC passes, made on the GPU box (the
# raw rocprofv3 CSVs exceed gpurun's 64 MiB copy-back), then the raw per-dispatch
# CSVs removed; the summaries go to gpurun_out/<name>/summ/ for profiles/<round>/.
#   bash tools/collect_profiles.sh <name>
set -o pipefail
D=gpurun_out/${1:?name}
S=$D/summ
mkdir -p $S
[ -f $D/syrk_timed_launches.json ] && cp $D/syrk_timed_launches.json $S/syrk_timed_launches_trace.json
[ -f $D/prof_dense/run_kernel_stats.csv ] && cp $D/prof_dense/run_kernel_stats.csv $S/rocprof_kernel_stats_dense_timed.csv
[ -f $D/bench_dense_under_rocprof.json ] && cp $D/bench_dense_under_rocprof.json $S/
[ -f $D/band_timeline.txt ] && cp $D/band_timeline.txt $S/
[ -f $D/prof_band/run_kernel_stats.csv ] && cp $D/prof_band/run_kernel_stats.csv $S/rocprof_kernel_stats_band.csv
for c in sparse4 sparse5; do
  [ -f $D/spmm_timed_launches_$c.json ] && cp $D/spmm_timed_launches_$c.json $S/
  [ -f $D/prof_$c/run_kernel_stats.csv ] && cp $D/prof_$c/run_kernel_stats.csv $S/rocprof_kernel_stats_$c.csv
  [ -f $D/bench_under_rocprof_$c.json ] && cp $D/bench_under_rocprof_$c.json $S/
  if [ -d $D/pmc_${c}_FETCH_SIZE ]; then
    PMC_MARKS=1 python tools/pmc_summary.py $S/pmc_traffic_$c.json "bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline (assembly, reference checks, one timed step between timing marks, isolated launches); FETCH_SIZE / WRITE_SIZE passes (KB; gfx950 FETCH counts half of wide streaming reads); per_dispatch_timed = the timed step's dispatches (first pair of timing_mark_kernel)" $D/pmc_${c}_FETCH_SIZE $D/pmc_${c}_WRITE_SIZE > /dev/null || exit 1
  fi
done
if [ -d $D/pmc_dense_FETCH_SIZE ]; then
  PMC_FIRST=127 python tools/pmc_summary.py $S/pmc_traffic_outer16_b64.json "bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-band --no-sparse --no-timing (batch 64, outer panel 16), FETCH_SIZE / WRITE_SIZE passes (KB); per_dispatch_first = the timed step's 127 batch-64 syrk launches" $D/pmc_dense_FETCH_SIZE $D/pmc_dense_WRITE_SIZE > /dev/null || exit 1
fi
if [ -d $D/pmc_mfma ]; then
  python tools/pmc_summary.py $S/pmc_dense_mfma.json "dense line, one 64-eta step: MFMA busy / fp64 MOPS / CU busy / GRBM_GUI_ACTIVE" $D/pmc_mfma > /dev/null || exit 1
fi
if [ -d $D/pmc_band_mfma ]; then
  python tools/pmc_summary.py $S/pmc_band_mfma.json "tools/band_refresh_probe.py 128 1: two band reductions (N = 16384); MFMA busy / fp64 MOPS / CU busy / GRBM_GUI_ACTIVE" $D/pmc_band_mfma > /dev/null || exit 1
fi
if [ -d $D/pmc_band_FETCH_SIZE ]; then
  python tools/pmc_summary.py $S/pmc_band_traffic.json "tools/band_refresh_probe.py 128 1: two band reductions (N = 16384); FETCH_SIZE / WRITE_SIZE passes (KB; gfx950 FETCH counts half of wide streaming reads)" $D/pmc_band_FETCH_SIZE $D/pmc_band_WRITE_SIZE > /dev/null || exit 1
fi
find $D -name '*kernel_trace.csv' -delete
find $D -name '*counter_collection.csv' -delete
ls -la $S
