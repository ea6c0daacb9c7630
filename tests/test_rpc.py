"""paddle.distributed.rpc (distributed/rpc over the TensorPipe agent) on CPU: the reference's
docstring examples (python/paddle/distributed/rpc/rpc.py:73-369) at world 1, and two workers
calling each other's functions (sync, async, kwargs, exceptions, worker infos)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def add(a, b):
    return a + b


def scale(x, k=1):
    return x * k


def boom():
    raise ValueError("boom from the callee")


def test_rpc_world1():
    from paddle_ray_amd.distributed import rpc
    os.environ['PADDLE_WORKER_ENDPOINT'] = '127.0.0.1:9002'
    try:
        rpc.init_rpc("worker0", rank=0, world_size=1, master_endpoint="127.0.0.1:%d" % _port())
        assert rpc.rpc_sync("worker0", add, args=(2, 3)) == 5
        assert rpc.rpc_async("worker0", add, args=(2, 3)).wait() == 5
        info = rpc.get_worker_info("worker0")
        assert str(info) == "{name: worker0, rank: 0, ip: 127.0.0.1, port: 9002}"
        assert rpc.get_all_worker_infos() == [info] and rpc.get_current_worker_info() == info
        rpc.shutdown()
    finally:
        os.environ.pop('PADDLE_WORKER_ENDPOINT', None)


def _worker(rank, port, q):
    from paddle_ray_amd.distributed import rpc
    os.environ['PADDLE_TRAINER_ID'] = str(rank)
    os.environ['PADDLE_TRAINERS_NUM'] = '2'
    os.environ['PADDLE_MASTER_ENDPOINT'] = '127.0.0.1:%d' % port
    os.environ['PADDLE_WORKER_ENDPOINT'] = '127.0.0.1:%d' % (9100 + rank)
    rpc.init_rpc("w%d" % rank)
    other = "w%d" % (1 - rank)
    out = {'sync': rpc.rpc_sync(other, add, args=(rank, 10)),
           'kw': rpc.rpc_async(other, scale, args=(3,), kwargs={'k': 4}).wait(),
           'infos': [str(i) for i in rpc.get_all_worker_infos()]}
    try:
        rpc.rpc_sync(other, boom)
        out['err'] = None
    except Exception as e:  # the callee's exception re-raised here
        out['err'] = 'boom from the callee' in str(e)
    rpc.shutdown()
    q.put((rank, out))


def test_rpc_two_workers():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_infos = ["{name: w0, rank: 0, ip: 127.0.0.1, port: 9100}", "{name: w1, rank: 1, ip: 127.0.0.1, port: 9101}"]
    for r in range(2):
        assert res[r]['sync'] == r + 10 and res[r]['kw'] == 12
        assert res[r]['infos'] == want_infos and res[r]['err'] is True


def test_rpc_requires_init():
    from paddle_ray_amd.distributed import rpc
    with pytest.raises(RuntimeError):
        rpc.get_current_worker_info()
