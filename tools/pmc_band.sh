set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r2pmc/pmc_band_mfma -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1 > gpurun_out/r2pmc/pmc_band_mfma.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r2pmc/pmc_band_fetch -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1 > gpurun_out/r2pmc/pmc_band_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r2pmc/pmc_band_write -o run --output-format csv -- python3 tools/band_refresh_probe.py 128 1 > gpurun_out/r2pmc/pmc_band_write.log 2>&1
