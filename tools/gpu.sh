# One GPU driver for gpurun (replaces the round-1..3 one-off gpu_*.sh scripts).
#   bash tools/gpu.sh <name> <task> [<task> ...]
# Logs and results go to gpurun_out/<name>/. Every GPU step runs under its own
# timeout; the first failing step ends the call (no retries).
# Tasks:
#   tests        -m gpu suite (verbose log) + smoke()
#   tests:<expr> -m gpu tests matching -k <expr>
#   bench        default bench line (dense + band + sparse + CPU baselines)
#   bench-fast   default bench line without CPU baselines
#   sparse4 / sparse5   bench --config sparseN (with its CPU baseline)
#   rehearse     N=2 ranks on the shared device (gloo): dense+band+sparse line,
#                and the N=1 line with an RCCL process group (GPMI_BENCH_PG=1)
#   trace        rocprofv3 --kernel-trace --stats of bench --steps 3 --warmup 1
#                --no-cpu-baseline (dense+band+sparse) + the bench line it ran
#   trace-dense  the same for the dense line only (--no-band --no-sparse): the
#                headline syrk_kernel launches, summarised by tools/trace_summary.py
#   pmc-dense    FETCH_SIZE / WRITE_SIZE passes over the dense line (batch 64)
#   pmc-mfma     MFMA busy / fp64 MOPS / CU busy / GPU clock pass over the dense line
#   pmc-band     the same MFMA pass and FETCH / WRITE passes over two band reductions
#                (tools/band_refresh_probe.py 128 1)
#   pmc-sparse4 / pmc-sparse5   FETCH / WRITE passes over one sparse step
#   trace-sparse4 / trace-sparse5   kernel-trace stats of bench --config sparseN
#   trace-band   kernel trace of two band reductions + the per-panel timeline
#                (tools/band_timeline.py)
#   host         the box's CPU / cgroup facts (host.txt)
#   py:<file>[:<arg>]   python -u <file> [<arg>] (a probe under tools/)
#   trace-py:<file>[:<arg>]   the same under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
NAME=${1:?name}
shift
D=gpurun_out/$NAME
mkdir -p $D

run() {  # run <seconds> <log> <cmd...>
  local t=$1 logf=$2
  shift 2
  echo "[gpu.sh] $* (limit ${t}s) -> $logf"
  timeout -k 10 $t "$@" > $logf 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] FAILED rc=$rc: $*"
    tail -40 $logf
    exit $rc
  fi
}

for task in "$@"; do
  case $task in
    tests)
      run 1100 $D/tests.log python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
      tail -1 $D/tests.log
      run 200 $D/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
      tail -1 $D/smoke.log ;;
    tests:*)
      run 900 $D/tests_k.log python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -k "${task#tests:}"
      tail -1 $D/tests_k.log ;;
    bench)
      run 900 $D/bench.err python -u bench.py --out-json $D/bench.json
      python tools/bench_summary.py $D/bench.json ;;
    bench-fast)
      run 900 $D/bench_fast.err python -u bench.py --no-cpu-baseline --out-json $D/bench_fast.json
      python tools/bench_summary.py $D/bench_fast.json ;;
    sparse4|sparse5)
      run 400 $D/$task.err python -u bench.py --config $task --out-json $D/$task.json
      python tools/bench_summary.py $D/$task.json ;;
    rehearse)
      GPMI_BENCH_SHARE_DEVICE=1 GPMI_BENCH_BACKEND=gloo \
        run 900 $D/n2.err python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --out-json $D/n2.json
      python tools/bench_summary.py $D/n2.json
      GPMI_BENCH_PG=1 run 900 $D/pg1.err python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --out-json $D/pg1.json
      python tools/bench_summary.py $D/pg1.json ;;
    trace)
      run 900 $D/trace.err rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --out-json $D/bench_under_rocprof.json
      python tools/bench_summary.py $D/bench_under_rocprof.json ;;
    trace-dense)
      run 600 $D/trace_dense.err rocprofv3 --kernel-trace --stats -d $D/prof_dense -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-band --no-sparse --no-extras --out-json $D/bench_dense_under_rocprof.json
      python tools/trace_summary.py --timed-syrk $D/prof_dense $D/bench_dense_under_rocprof.json > $D/syrk_timed_launches.json
      cat $D/syrk_timed_launches.json ;;
    pmc-dense)
      for c in FETCH_SIZE WRITE_SIZE; do
        run 300 $D/pmc_$c.log rocprofv3 --pmc $c --kernel-trace -d $D/pmc_dense_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-band --no-sparse --no-timing
      done ;;
    pmc-mfma)
      run 300 $D/pmc_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d $D/pmc_mfma -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band --no-sparse ;;
    pmc-peak)
      # the fp64 MFMA microbenchmark (tools/fp64_peak, built in the container) under
      # the same MFMA-busy / clock counters as pmc-mfma: the ceiling's own busy fraction
      run 120 $D/fp64_peak_plain.log ./tools/fp64_peak
      cat $D/fp64_peak_plain.log
      run 200 $D/pmc_peak.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d $D/pmc_peak -o run --output-format csv -- ./tools/fp64_peak
      python tools/pmc_summary.py $D/pmc_peak.json "fp64_peak under MFMA counters" $(dirname $(find $D/pmc_peak -name "*counter_collection.csv")) > /dev/null && cat $D/pmc_peak.json ;;
    pmc-band)
      run 200 $D/pmc_band_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d $D/pmc_band_mfma -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1
      for c in FETCH_SIZE WRITE_SIZE; do
        run 200 $D/pmc_band_$c.log rocprofv3 --pmc $c --kernel-trace -d $D/pmc_band_$c -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1
      done ;;
    pmc-sparse4|pmc-sparse5)
      cfg=${task#pmc-}
      for c in FETCH_SIZE WRITE_SIZE; do
        run 200 $D/pmc_${cfg}_$c.log rocprofv3 --pmc $c --kernel-trace -d $D/pmc_${cfg}_$c -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline
      done ;;
    trace-band)
      run 300 $D/trace_band.err rocprofv3 --kernel-trace --stats -d $D/prof_band -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1
      python tools/band_timeline.py $D/prof_band 10 60 110 > $D/band_timeline.txt
      head -12 $D/band_timeline.txt ;;
    trace-sparse4|trace-sparse5)
      cfg=${task#trace-}
      run 400 $D/trace_$cfg.err rocprofv3 --kernel-trace --stats -d $D/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --out-json $D/bench_under_rocprof_$cfg.json
      python tools/bench_summary.py $D/bench_under_rocprof_$cfg.json
      python tools/trace_summary.py --timed-spmm $D/prof_$cfg $D/bench_under_rocprof_$cfg.json > $D/spmm_timed_launches_$cfg.json
      cat $D/spmm_timed_launches_$cfg.json ;;
    host)
      (nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print('aff', len(os.sched_getaffinity(0)), 'omp', os.environ.get('OMP_NUM_THREADS'))"; lscpu | head -20) > $D/host.txt 2>&1 ;;
    trace-py:*)
      # trace-py:<file>[:<arg>]: kernel-trace stats of a probe under tools/
      spec=${task#trace-py:}
      f=${spec%%:*}
      arg=""
      [ "$spec" != "$f" ] && arg=${spec#*:}
      b=$(basename $f .py)
      run 600 $D/trace_$b.log rocprofv3 --kernel-trace --stats -d $D/prof_$b -o run --output-format csv -- python3 -u $f $arg
      tail -12 $D/trace_$b.log ;;
    py:*)
      # py:<file>[:<arg>]
      spec=${task#py:}
      f=${spec%%:*}
      arg=""
      [ "$spec" != "$f" ] && arg=${spec#*:}
      run 900 $D/$(basename $f .py)$arg.log python -u $f $arg
      tail -30 $D/$(basename $f .py)$arg.log ;;
    *)
      echo "[gpu.sh] unknown task $task"; exit 2 ;;
  esac
done
echo "[gpu.sh] done: $*"
