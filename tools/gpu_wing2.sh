# Window SpMM default at HEAD: sparse GPU tests, both sparse bench lines, and the
# FETCH_SIZE / WRITE_SIZE passes whose last 50 s=20 dispatches the bench's
# roofline.traffic reads (profiles/r3/pmc_traffic_sparse{4,5}.json).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/wing2
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_dense_slq.py -q -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python -u bench.py --config $cfg > $D/bench_$cfg.json 2> $D/bench_$cfg.err || { tail -5 $D/bench_$cfg.err; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $D/pmc_${cfg}_$c -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline > $D/pmc_${cfg}_$c.log 2>&1 || exit 1
  done
  echo "$cfg ok"
done
