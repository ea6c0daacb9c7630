import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _parse(argv=None):
    p = argparse.ArgumentParser('paddle_ray_amd.distributed.launch')
    p.add_argument('--gpus', '--devices', dest='devices', default=None)
    p.add_argument('--nproc_per_node', type=int, default=None)
    p.add_argument('--master', default=None)
    p.add_argument('--nnodes', default='1')
    p.add_argument('--rank', type=int, default=0)
    p.add_argument('--log_dir', default='log')
    p.add_argument('--job_id', default='default')
    # elastic parameters (reference launch/context/args_envs.py:163-186; env PADDLE_MAX_RESTART,
    # PADDLE_ELASTIC_LEVEL, PADDLE_ELASTIC_TIMEOUT): level -1 = no restart (a failed rank ends the
    # job), 0 = failed exit, 1 = internal restart of the whole pod up to max_restart times
    p.add_argument('--max_restart', type=int, default=int(os.environ.get('PADDLE_MAX_RESTART', '3')))
    p.add_argument('--elastic_level', type=int, default=int(os.environ.get('PADDLE_ELASTIC_LEVEL', '-1')))
    p.add_argument('--elastic_timeout', type=int, default=int(os.environ.get('PADDLE_ELASTIC_TIMEOUT', '30')))
    p.add_argument('training_script')
    p.add_argument('training_script_args', nargs=argparse.REMAINDER)
    return p.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_pod(a, devs, addr, port, restart):
    """Start one process per device and watch them: 0 when all exit cleanly, else the first
    failing rank's exit code (the other ranks are terminated)."""
    n = len(devs)
    procs = []
    eps = ','.join(f'{addr}:{int(port) + i}' for i in range(n))
    for r, d in enumerate(devs):
        env = dict(os.environ)
        env.update({'RANK': str(r), 'LOCAL_RANK': str(r), 'WORLD_SIZE': str(n),
                    'MASTER_ADDR': addr, 'MASTER_PORT': str(port),
                    'PADDLE_TRAINER_ID': str(r), 'PADDLE_TRAINERS_NUM': str(n),
                    'PADDLE_TRAINER_ENDPOINTS': eps, 'PADDLE_CURRENT_ENDPOINT': eps.split(',')[r],
                    'PADDLE_JOB_ID': a.job_id, 'PADDLE_RESTART_COUNT': str(restart),
                    'FLAGS_selected_gpus': str(d)})
        log = open(os.path.join(a.log_dir, f'workerlog.{r}'), 'a' if restart else 'w')
        cmd = [sys.executable, '-u', a.training_script] + a.training_script_args
        procs.append((subprocess.Popen(cmd, env=env, stdout=log if r else None,
                                       stderr=subprocess.STDOUT if r else None), log))
    code = 0
    try:
        while procs:
            for p, log in list(procs):
                rc = p.poll()
                if rc is None:
                    continue
                procs.remove((p, log))
                log.close()
                if rc != 0 and code == 0:
                    code = rc
                    for q, _ in procs:  # a failed rank takes the pod down
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for q, _ in procs:
            q.send_signal(signal.SIGTERM)
        for q, _ in procs:
            q.wait()
        raise
    return code


def _multi_node(a):
    n = str(a.nnodes or '1')
    try:
        hi = int(n.split(':')[-1])
    except ValueError:
        hi = 1
    return hi > 1


def launch(argv=None):
    a = _parse(argv)
    if a.devices:
        devs = [d for d in a.devices.split(',') if d != '']
    else:
        n = a.nproc_per_node or int(os.environ.get('PRA_NPROC', '1'))
        devs = [str(i) for i in range(n)]
    os.makedirs(a.log_dir, exist_ok=True)
    restart = 0
    while True:
        if a.master:
            addr, port = a.master.split(':')
        else:   # a fresh port per attempt (the previous pod's may still be in TIME_WAIT)
            addr, port = '127.0.0.1', str(_free_port())
        try:
            code = _run_pod(a, devs, addr, port, restart)
        except KeyboardInterrupt:
            sys.exit(130)
        # reference controllers/collective.py:208: the pod is rebuilt while restart <= max_restart
        if code == 0 or a.elastic_level < 1 or restart >= a.max_restart:
            sys.exit(code)
        if _multi_node(a):
            # the other nodes' pods keep their rendezvous: rebuilding only this one would hang at
            # init. A multi-node restart needs the peers restarted too (the reference coordinates
            # it through its master store); report and exit with the failure instead
            print(f'[launch] job {a.job_id}: a rank exited with {code}; in-place restart is '
                  f'single-node only (--nnodes {a.nnodes}): not restarting', file=sys.stderr, flush=True)
            sys.exit(code)
        restart += 1
        print(f'[launch] job {a.job_id}: a rank exited with {code}; restart {restart}/{a.max_restart}',
              file=sys.stderr, flush=True)
