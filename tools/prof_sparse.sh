set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in sparse4 sparse5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$cfg.log 2>&1 || exit 1
  echo "$cfg ok"
done
