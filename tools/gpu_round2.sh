# band tests incl. cyclic-reduction derivative terms + timings, then the full pass
bash tools/gpu_bcr.sh ${1:-r}_bcr && bash tools/gpu_round.sh ${1:-r}
