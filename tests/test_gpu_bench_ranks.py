"""bench.py at N = 2 ranks on the one-GPU box: ``python bench.py --gpus 2``
launches the two ranks itself, both share device 0 (GPMI_BENCH_SHARE_DEVICE=1)
and use gloo for the collectives (RCCL refuses two ranks on one device). The
line must report two ranks and the same curve as the N = 1 run."""

import json
import os
import subprocess
import sys

import numpy
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, 'bench.py')
ARGS = ['--grid', '32', '--steps', '1', '--warmup', '1', '--no-band', '--no-sparse',
        '--no-cpu-baseline']


def _run(gpus, extra_env):
    env = dict(os.environ, **extra_env)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    out = subprocess.run([sys.executable, '-u', BENCH, '--gpus', str(gpus)] + ARGS, env=env,
                         capture_output=True, text=True, timeout=240, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_on_shared_device_equal_one_rank():
    one = _run(1, {})
    two = _run(2, {'GPMI_BENCH_SHARE_DEVICE': '1', 'GPMI_BENCH_BACKEND': 'gloo'})
    assert one['n_gpus'] == 1 and two['n_gpus'] == 2
    assert [d['rank'] for d in two['devices']] == [0, 1]
    assert all(d['shared_device'] and d['device'] == 0 for d in two['devices'])
    assert two['config']['eta_per_rank_per_step'] == 32
    # the lp of the gathered curve's first eta equals the N = 1 line's
    a, b = numpy.asarray(one['lp_sample']), numpy.asarray(two['lp_sample'])
    assert a[0] == b[0]
    numpy.testing.assert_allclose(b, a, rtol=1e-12)
