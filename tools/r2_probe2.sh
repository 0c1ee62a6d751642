set -o pipefail
mkdir -p gpurun_out/r2
for v in "" mp1 mp2 mnt0; do GPMI_LIB_VARIANT=$v timeout -k 10 120 python -u tools/asm_probe.py || exit 1; done > gpurun_out/r2/asm_probe.txt
cat gpurun_out/r2/asm_probe.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
GPMI_LZ_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_lz1 -o run -- python -u bench.py --config sparse4 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r2/prof_lz1.json 2>gpurun_out/r2/prof_lz1.err
