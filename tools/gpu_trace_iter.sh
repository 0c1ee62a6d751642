# kernel traces: sparse5 bench step, band reduction probe at delay 1 and 4
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-tr}
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_sparse5 -o run --output-format csv -- python3 bench.py --config sparse5 --steps 3 --warmup 1 --no-cpu-baseline > $D/bench_sparse5.json 2> $D/bench_sparse5.err || exit 1
for dl in 1 4; do
  GPMI_BAND_DELAY=$dl timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_band_d$dl -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1 > $D/band_d$dl.log 2>&1 || exit 1
done
echo done
