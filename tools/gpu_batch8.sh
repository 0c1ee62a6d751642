set -o pipefail
mkdir -p gpurun_out/b8
for g in 0 1; do GPMI_GROUPS=$g timeout -k 10 300 python3 tools/batch8_probe.py > gpurun_out/b8/g$g.txt 2>&1 || { tail -5 gpurun_out/b8/g$g.txt; exit 1; }; cat gpurun_out/b8/g$g.txt; done
