set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in sparse4 sparse5; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${cfg}_fetch -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_${cfg}_fetch.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_${cfg}_write -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_${cfg}_write.log 2>&1 || exit 1
  echo "$cfg ok"
done
