#!/bin/bash
# Rehearse the N>1 bench flow on the one-GPU box: two ranks share device 0 and
# use gloo for the barrier / max-time all-reduce / all-gather (RCCL refuses two
# ranks on one device). Numbers are not scaling data; the JSON shape and the
# gathered curves are what this checks.
set -o pipefail
mkdir -p gpurun_out/n2
export GPMI_BENCH_BACKEND=gloo GPMI_BENCH_SHARE_DEVICE=1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 \
    > gpurun_out/n2/dense.json 2> gpurun_out/n2/dense.log &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 \
    --config sparse4 > gpurun_out/n2/sparse4.json 2> gpurun_out/n2/sparse4.log &&
cat gpurun_out/n2/dense.json gpurun_out/n2/sparse4.json
