# The sparse GPU tests, then tools/shard_probe.py for configs 4 and 5: rank 0's
# device work of an N-rank sparse step (N = 1, 2, 4, 8) on one GPU.
#   bash tools/shard_ab.sh <name>
set -o pipefail
D=gpurun_out/${1:?name}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_dense_slq.py -x -q --timeout 300 --timeout-method thread > $D/sparse_tests.log 2>&1 || { tail -30 $D/sparse_tests.log; exit 1; }
tail -1 $D/sparse_tests.log
for cfg in sparse4 sparse5; do
  timeout -k 10 400 python -u tools/shard_probe.py $cfg 5 > $D/shard_probe_$cfg.log 2>&1 || { tail -20 $D/shard_probe_$cfg.log; exit 1; }
  grep rank0 $D/shard_probe_$cfg.log | head -4
done
