"""paddle.distributed.spawn (parity: python/paddle/distributed/spawn.py).

Starts ``nprocs`` worker processes (one per GPU) with the torch.distributed
rendezvous env set (127.0.0.1), runs ``func(*args)`` in each, joins them.
"""
import multiprocessing as mp
import os
import socket


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, nprocs, port, func, args, env):
    os.environ.update(env)
    os.environ.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(nprocs),
                       'PADDLE_TRAINER_ID': str(rank), 'PADDLE_TRAINERS_NUM': str(nprocs),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    func(*args)


class MultiprocessContext:
    def __init__(self, procs):
        self.processes = procs

    def join(self, timeout=None):
        """Poll every worker; the first failure terminates the others (a dead rank would
        otherwise leave its peers blocked in a collective until the comm timeout)."""
        import time
        t_end = None if timeout is None else time.monotonic() + timeout
        live = list(self.processes)
        failed = False
        while live:
            for p in list(live):
                if p.exitcode is not None:
                    live.remove(p)
                    failed = failed or p.exitcode != 0
            if live and (failed or (t_end is not None and time.monotonic() > t_end)):
                for p in live:
                    p.terminate()
                for p in live:
                    p.join(10)
                    if p.exitcode is None:
                        p.kill()
                        p.join()
                if not failed:
                    return False
                break
            time.sleep(0.1)
        ok = all(p.exitcode == 0 for p in self.processes)
        if not ok:
            codes = [p.exitcode for p in self.processes]
            raise RuntimeError(f"spawned workers failed with exit codes {codes}")
        return True


def spawn(func, args=(), nprocs=-1, join=True, daemon=False, **options):
    if nprocs <= 0:
        import torch
        nprocs = max(torch.cuda.device_count(), 1)
    port = options.get('port', _free_port())
    ctx = mp.get_context('spawn')
    env = {k: v for k, v in os.environ.items() if k.startswith(('PRA_', 'FLAGS_', 'HSA_'))}
    procs = []
    for r in range(nprocs):
        p = ctx.Process(target=_worker, args=(r, nprocs, port, func, tuple(args), env),
                        daemon=daemon)
        p.start()
        procs.append(p)
    c = MultiprocessContext(procs)
    if join:
        c.join()
    return c
