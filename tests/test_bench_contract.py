"""The driver's bench.py contract on the CPU (gloo): launched by torch.distributed.run with one
process per rank, or self-spawning its ranks from ``--gpus N``, bench.py prints exactly ONE JSON
line (rank 0) with the whole-job value, n_gpus = N, and ZeRO-3 active at N > 1."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ['--steps', '1', '--warmup', '1', '--model', 'gpt3-tiny', '--micro-batch', '2', '--seq', '64']


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith('{')]


def _env():
    env = dict(os.environ, OMP_NUM_THREADS='2', PRA_BENCH_TIMEOUT='200')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    return env


def _check(lines, n):
    assert len(lines) == 1, lines
    r = lines[0]
    assert r['n_gpus'] == n and r['steps'] == 1 and r['warmup'] == 1
    assert r['value'] > 0 and r['ms_per_step'] > 0 and r['higher_is_better'] is True
    assert r['config']['global_batch'] == 2 * n
    assert r['config']['zero3_active'] is (n > 1)
    return r


@pytest.mark.timeout(300)
def test_bench_under_torchrun_two_ranks():
    # (--standalone: torchrun picks a free rendezvous port itself, no race with parallel tests)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--standalone', '--local-addr', '127.0.0.1',
           '--nnodes=1', '--nproc-per-node', '2', 'bench.py', '--gpus', '2'] + ARGS
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    _check(_json_lines(p.stdout), 2)


@pytest.mark.timeout(300)
def test_bench_self_spawned_ranks():
    p = subprocess.run([sys.executable, 'bench.py', '--gpus', '2'] + ARGS, cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    _check(_json_lines(p.stdout), 2)


@pytest.mark.timeout(300)
def test_bench_single_rank_defaults_shape():
    p = subprocess.run([sys.executable, 'bench.py'] + ARGS, cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    r = _check(_json_lines(p.stdout), 1)
    assert r['dtype'] == 'bf16' and r['scaling'] == 'weak' and 'synthetic' in r['data']
