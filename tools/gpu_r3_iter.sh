# sparse iteration, then the band delayed-update iteration (one gpurun call)
bash tools/gpu_sparse_iter.sh ${1:-it}_sp && bash tools/gpu_band_delay.sh ${1:-it}_bd
