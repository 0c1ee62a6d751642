set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 2; do
  GPMI_GROUPS=$g timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-band > gpurun_out/grp$g.log 2>&1 || exit 1
done
GPMI_GROUPS=2 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-band --eta-per-rank 32 > gpurun_out/grp2_32.log 2>&1
