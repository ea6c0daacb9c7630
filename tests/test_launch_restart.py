"""paddle_ray_amd.distributed.launch: a failed rank takes the pod down; with --elastic_level 1 the
pod is rebuilt up to --max_restart times (reference launch/controllers/collective.py:208), the
attempt number in PADDLE_RESTART_COUNT so a script can resume from its checkpoint."""
import os
import subprocess
import sys
import textwrap

SCRIPT = textwrap.dedent('''
    import os, sys
    r, n = int(os.environ['PADDLE_TRAINER_ID']), int(os.environ['PADDLE_TRAINERS_NUM'])
    k = int(os.environ['PADDLE_RESTART_COUNT'])
    with open(os.path.join(sys.argv[1], 'r%d_a%d' % (r, k)), 'w') as f:
        f.write(os.environ['PADDLE_TRAINER_ENDPOINTS'])
    if r == 1 and k < int(sys.argv[2]):
        import time
        t = time.time()   # fail only after rank 0 has recorded this attempt (no kill race)
        while not os.path.exists(os.path.join(sys.argv[1], 'r0_a%d' % k)) and time.time() - t < 30:
            time.sleep(0.05)
        sys.exit(3)
''')


def _run(tmp_path, fail_attempts, *flags):
    script = tmp_path / 'train.py'
    script.write_text(SCRIPT)
    out = tmp_path / 'out'
    out.mkdir(exist_ok=True)
    cmd = [sys.executable, '-m', 'paddle_ray_amd.distributed.launch', '--nproc_per_node', '2',
           '--log_dir', str(tmp_path / 'log'), *flags, str(script), str(out), str(fail_attempts)]
    env = dict(os.environ, PYTHONPATH=os.getcwd())
    rc = subprocess.run(cmd, env=env, timeout=120).returncode
    return rc, sorted(p.name for p in out.iterdir())


def test_failed_rank_ends_job_without_elastic(tmp_path):
    rc, files = _run(tmp_path, 1)
    assert rc == 3 and files == ['r0_a0', 'r1_a0']


def test_elastic_restart_recovers(tmp_path):
    rc, files = _run(tmp_path, 2, '--elastic_level', '1', '--max_restart', '3')
    assert rc == 0
    assert files == ['r0_a0', 'r0_a1', 'r0_a2', 'r1_a0', 'r1_a1', 'r1_a2']


def test_elastic_restart_budget(tmp_path):
    rc, files = _run(tmp_path, 5, '--elastic_level', '1', '--max_restart', '1')
    assert rc == 3 and files == ['r0_a0', 'r0_a1', 'r1_a0', 'r1_a1']
