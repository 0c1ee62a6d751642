# Round-3 evidence at HEAD: rocprofv3 kernel-trace stats of the default bench (dense,
# band, dense slq, sparse modes), and FETCH_SIZE / WRITE_SIZE passes over the
# dense_mm probe (dense 'slq' K X) and the sparse5 step (multi-shift CG change).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/ev
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/bench_under_rocprof.json 2> $D/bench_under_rocprof.err || { tail -5 $D/bench_under_rocprof.err; exit 1; }
echo "trace ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $D/pmc_mm_$c -o run --output-format csv -- python3 tools/dense_mm_probe.py > $D/pmc_mm_$c.log 2>&1 || exit 1
done
echo "pmc ok"
