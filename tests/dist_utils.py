"""Helpers to run a function on N gloo ranks (CPU) and collect per-rank numpy results."""
import os
import pickle
import socket
import sys
import traceback

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, outdir):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port),
                       'PRA_FORCE_CPU': '1'})
    sys.path.insert(0, ROOT)
    try:
        import paddle_ray_amd as paddle
        paddle.set_device('cpu')
        paddle.distributed.init_parallel_env(backend='gloo')
        res = fn(rank, world, *args)
        with open(os.path.join(outdir, f'r{rank}.pkl'), 'wb') as f:
            pickle.dump(res, f)
        paddle.distributed.barrier()
        paddle.distributed.destroy_process_group()
    except Exception:
        with open(os.path.join(outdir, f'r{rank}.err'), 'w') as f:
            f.write(traceback.format_exc())
        raise


def run_ranks(fn, world, tmpdir, args=()):
    port = _free_port()
    mp.start_processes(_entry, args=(world, port, fn, args, str(tmpdir)), nprocs=world,
                       join=True, start_method='spawn')
    out = []
    for r in range(world):
        p = os.path.join(str(tmpdir), f'r{r}.pkl')
        if not os.path.exists(p):
            err = open(os.path.join(str(tmpdir), f'r{r}.err')).read()
            raise RuntimeError(err)
        with open(p, 'rb') as f:
            out.append(pickle.load(f))
    return out
