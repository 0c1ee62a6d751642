# Re-entry check at HEAD: -m gpu suite, smoke(), and the driver's bench command timed.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r3b}
mkdir -p $D
bash tools/gpu_tests.sh ${1:-r3b} || exit 1
s=$(date +%s)
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver.json 2> $D/bench_driver.err || { tail -5 $D/bench_driver.err; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
