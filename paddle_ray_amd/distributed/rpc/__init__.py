"""paddle.distributed.rpc: named workers calling Python functions on each other.

Parity: python/paddle/distributed/rpc/rpc.py (init_rpc:73, rpc_sync:141, rpc_async:179,
shutdown:270, get_worker_info:299, get_all_worker_infos:328, get_current_worker_info:354) over
the reference's brpc agent (paddle/fluid/distributed/rpc/). Here the transport is PyTorch's
TensorPipe RPC agent (TCP/shared memory between hosts' CPUs; no GPU state crosses the wire unless
a tensor argument lives on the device). The rendezvous uses the reference's inputs: the worker's
rank / world size from the arguments or PADDLE_TRAINER_ID / PADDLE_TRAINERS_NUM, the master's
``ip:port`` from ``master_endpoint`` or PADDLE_MASTER_ENDPOINT; PADDLE_WORKER_ENDPOINT (or a free
local port) is the ``ip:port`` a WorkerInfo reports. Timeouts are in seconds; <= 0 waits forever
(the reference's default is -1).
"""
import os
import socket

import torch.distributed.rpc as _rpc

__all__ = ['init_rpc', 'shutdown', 'rpc_sync', 'rpc_async', 'get_worker_info', 'get_all_worker_infos',
           'get_current_worker_info', 'WorkerInfo']

_DEFAULT_RPC_TIMEOUT = -1
_STATE = {'self': None, 'infos': None}


class WorkerInfo:
    __slots__ = ('name', 'rank', 'ip', 'port')

    def __init__(self, name, rank, ip, port):
        self.name, self.rank, self.ip, self.port = name, int(rank), ip, int(port)

    def __repr__(self):
        return "{name: %s, rank: %d, ip: %s, port: %d}" % (self.name, self.rank, self.ip, self.port)

    __str__ = __repr__

    def __eq__(self, other):
        return isinstance(other, WorkerInfo) and (self.name, self.rank, self.ip, self.port) == (
            other.name, other.rank, other.ip, other.port)

    def __hash__(self):
        return hash((self.name, self.rank))


class FutureWrapper:
    """Result of rpc_async: ``wait()`` blocks and returns fn's value (or raises its exception)."""

    def __init__(self, fut):
        self._fut = fut

    def wait(self):
        return self._fut.wait()

    def done(self):
        return self._fut.done()


def _free_endpoint():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind(('127.0.0.1', 0))
        return '127.0.0.1:%d' % s.getsockname()[1]
    finally:
        s.close()


def _timeout_s(timeout):
    # torch: 0 = no timeout
    return 0 if timeout is None or timeout <= 0 else float(timeout)


def _self_endpoint():
    return _STATE['self']


def init_rpc(name, rank=None, world_size=None, master_endpoint=None):
    """Start this process's RPC worker ``name`` and wait until all ``world_size`` workers joined."""
    if _STATE['self'] is not None:
        raise RuntimeError("init_rpc: RPC is already initialized; call shutdown() first")
    rank = int(os.environ['PADDLE_TRAINER_ID']) if rank is None else int(rank)
    world_size = int(os.environ['PADDLE_TRAINERS_NUM']) if world_size is None else int(world_size)
    master_endpoint = master_endpoint if master_endpoint is not None else os.environ['PADDLE_MASTER_ENDPOINT']
    addr, port = master_endpoint.rsplit(':', 1)
    ep = os.getenv('PADDLE_WORKER_ENDPOINT') or _free_endpoint()
    ip, wport = ep.rsplit(':', 1)
    timeout = int(os.getenv('FLAGS_stop_check_timeout', '900'))
    opts = _rpc.TensorPipeRpcBackendOptions(init_method='tcp://%s:%d' % (addr, int(port)), rpc_timeout=timeout)
    _rpc.init_rpc(name, rank=rank, world_size=world_size, rpc_backend_options=opts)
    _STATE['self'] = (name, rank, ip, int(wport))
    _STATE['infos'] = None


def _infos():
    if _STATE['self'] is None:
        raise RuntimeError("rpc is not initialized: call init_rpc first")
    if _STATE['infos'] is None:
        me = _STATE['self']
        out = []
        for w in sorted(_rpc.api._get_current_rpc_agent().get_worker_infos(), key=lambda w: w.id):
            name, rank, ip, port = me if w.name == me[0] else _rpc.rpc_sync(w.name, _self_endpoint)
            out.append(WorkerInfo(name, rank, ip, port))
        _STATE['infos'] = out
    return _STATE['infos']


def rpc_sync(to, fn, args=None, kwargs=None, timeout=_DEFAULT_RPC_TIMEOUT):
    """Run ``fn(*args, **kwargs)`` on worker ``to`` and return its result (blocking)."""
    return _rpc.rpc_sync(to, fn, args=tuple(args or ()), kwargs=dict(kwargs or {}), timeout=_timeout_s(timeout))


def rpc_async(to, fn, args=None, kwargs=None, timeout=_DEFAULT_RPC_TIMEOUT):
    """Non-blocking rpc_sync: returns a FutureWrapper whose ``wait()`` gives the result."""
    return FutureWrapper(_rpc.rpc_async(to, fn, args=tuple(args or ()), kwargs=dict(kwargs or {}),
                                        timeout=_timeout_s(timeout)))


def shutdown():
    """Block until every worker reached shutdown and all outstanding calls finished, then stop."""
    if _STATE['self'] is None:
        return
    _rpc.shutdown(graceful=True)
    _STATE['self'] = _STATE['infos'] = None


def get_worker_info(name):
    for w in _infos():
        if w.name == name:
            return w
    raise ValueError("rpc: no worker named %r" % (name,))


def get_all_worker_infos():
    return list(_infos())


def get_current_worker_info():
    me = _STATE['self']
    if me is None:
        raise RuntimeError("rpc is not initialized: call init_rpc first")
    return WorkerInfo(*me)
