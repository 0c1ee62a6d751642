set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/cols
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_dense_slq.py -v -x --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for cfg in sparse5 sparse4; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 5 > $D/$cfg.json 2> $D/$cfg.err || { tail -5 $D/$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(d['value'],1), round(d['ms_per_step'],2), d['reference_check'].get('gram_rel_err'))"
done
export GPMI_BENCH_BACKEND=gloo GPMI_BENCH_SHARE_DEVICE=1
for cfg in sparse4 sparse5; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --config $cfg > $D/n2_$cfg.json 2> $D/n2_$cfg.log || { tail -20 $D/n2_$cfg.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/n2_$cfg.json').read().strip().splitlines()[-1]);print('n2 $cfg', round(d['value'],1), d['n_gpus'], d['lp_sample'], d.get('reference_check'))"
done
