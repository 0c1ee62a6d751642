set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/lz
mkdir -p $D
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 tools/lanczos_probe.py sparse5 > $D/lz.txt 2>&1 || { tail -5 $D/lz.txt; exit 1; }
grep lanczos $D/lz.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof5 -o run --output-format csv -- python3 bench.py --config sparse5 --steps 3 --warmup 1 --no-cpu-baseline > $D/b5.json 2> $D/b5.err || { tail -5 $D/b5.err; exit 1; }
echo done
