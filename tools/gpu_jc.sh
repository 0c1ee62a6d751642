set -o pipefail
for v in "" jc8 jc24; do echo "variant=$v"; GPMI_LIB_VARIANT=$v timeout -k 10 200 python3 tools/lanczos_probe.py sparse5 2>&1 | grep lanczos || exit 1; done
