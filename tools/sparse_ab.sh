# A/B of the sparse lines on one box: bench --config sparse4 / sparse5 (no CPU
# baseline, 20 steps), the default build's path, then the same with the given
# environment assignments (e.g. GPMI_SPMM_WING=0), each under its own time limit.
#   bash tools/sparse_ab.sh <name> [VAR=value ...]
set -o pipefail
D=gpurun_out/${1:?name}
shift
mkdir -p $D
for cfg in sparse4 sparse5; do
  for side in a b; do
    if [ $side = b ]; then [ $# -gt 0 ] || continue; envs="$*"; else envs=""; fi
    env $envs timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 3 \
      --out-json $D/${cfg}_$side.json > $D/${cfg}_$side.err 2>&1 || { echo "FAILED $cfg $side"; tail -30 $D/${cfg}_$side.err; exit 1; }
    echo "[$cfg $side: ${envs:-default}]"
    python tools/bench_summary.py $D/${cfg}_$side.json | head -2
  done
done
