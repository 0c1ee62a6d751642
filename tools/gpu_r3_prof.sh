# Round-3 profiling pass: sparse step kernel traces (sparse4, sparse5) and the
# dense SYRK FETCH_SIZE / WRITE_SIZE PMC passes at HEAD (batch 64, outer 16).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r3prof}
mkdir -p $D
for cfg in sparse5 sparse4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $D/bench_prof_$cfg.json 2> $D/bench_prof_$cfg.err || exit 1
  echo "$cfg trace ok"
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/pmc_dense_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band > $D/pmc_dense_fetch.log 2>&1 || exit 1
echo "fetch ok"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/pmc_dense_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --no-band > $D/pmc_dense_write.log 2>&1 || exit 1
echo "write ok"
