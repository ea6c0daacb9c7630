"""Collective communication API (parity: python/paddle/distributed/collective.py,
python/paddle/distributed/communication/*.py, python/paddle/distributed/parallel.py:init_parallel_env).

One process per GPU; backend "nccl" == RCCL over xGMI on MI355X, "gloo" on CPU.
All collectives accept ``sync_op`` (paddle) and return a task with ``wait()``;
async tasks order the current HIP stream after the RCCL stream on ``wait()``
without blocking the host.
"""
import datetime
import os
import pickle

import numpy as np
import torch
import torch.distributed as dist

from . import watchdog as _watchdog

from ..framework.core import Tensor, _u, _default_device


class ReduceOp:
    SUM = 0
    MAX = 1
    MIN = 2
    PROD = 3
    AVG = 4


def _op(op):
    return {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.MAX: dist.ReduceOp.MAX,
            ReduceOp.MIN: dist.ReduceOp.MIN, ReduceOp.PROD: dist.ReduceOp.PRODUCT,
            ReduceOp.AVG: dist.ReduceOp.AVG}.get(op, op)


class Group:
    """paddle Group: global ``ranks`` list + this process's rank in it."""

    def __init__(self, ranks, pg=None, gid=0, name=None):
        self.ranks = list(ranks)
        self.process_group = pg
        self.id = gid
        self.name = name
        gr = dist.get_rank() if dist.is_initialized() else 0
        self.rank = self.ranks.index(gr) if gr in self.ranks else -1
        self.nranks = len(self.ranks)
        self.world_size = self.nranks

    def is_member(self):
        return self.rank >= 0

    def get_group_rank(self, rank):
        return self.ranks.index(rank) if rank in self.ranks else -1

    def __repr__(self):
        return f'Group(id={self.id}, ranks={self.ranks}, rank={self.rank})'


_groups = {}
_default_group = [None]
_group_counter = [1]


class ParallelEnv:
    def __init__(self):
        self._rank = int(os.environ.get('PADDLE_TRAINER_ID', os.environ.get('RANK', 0)))
        self._world_size = int(os.environ.get('PADDLE_TRAINERS_NUM',
                                              os.environ.get('WORLD_SIZE', 1)))
        self._local_rank = int(os.environ.get('LOCAL_RANK', self._rank))
        sel = os.environ.get('FLAGS_selected_gpus', '').split(',')[0].strip()
        self._device_id = int(sel) if sel.lstrip('-').isdigit() else self._local_rank
        eps = os.environ.get('PADDLE_TRAINER_ENDPOINTS', '')
        self._trainer_endpoints = eps.split(',') if eps else []
        self._current_endpoint = os.environ.get('PADDLE_CURRENT_ENDPOINT', '')

    @property
    def rank(self):
        return self._rank

    @property
    def world_size(self):
        return self._world_size

    @property
    def local_rank(self):
        return self._local_rank

    @property
    def device_id(self):
        return self._device_id

    @property
    def dev_id(self):
        return self._device_id

    @property
    def nranks(self):
        return self._world_size

    @property
    def trainer_endpoints(self):
        return self._trainer_endpoints

    @property
    def current_endpoint(self):
        return self._current_endpoint


def is_available():
    return dist.is_available()


def is_initialized():
    return dist.is_initialized()


def _bound_device(env=None):
    """The HIP device this rank drives: ``FLAGS_selected_gpus`` (set per rank by
    ``distributed.launch --gpus 4,5``) when present, else ``LOCAL_RANK`` — both modulo the
    visible device count (a rehearsal with more ranks than GPUs shares devices)."""
    env = env or ParallelEnv()
    n = max(torch.cuda.device_count(), 1)
    sel = os.environ.get('FLAGS_selected_gpus', '').split(',')[0].strip()
    if sel.lstrip('-').isdigit():
        return int(sel) % n
    return env.local_rank % n


def init_parallel_env(backend=None, timeout_s=None):
    """Create the default process group from torchrun / paddle launch env vars."""
    if dist.is_initialized():
        return _get_default_group()
    env = ParallelEnv()
    ws = env.world_size
    if 'MASTER_ADDR' not in os.environ:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
    if 'MASTER_PORT' not in os.environ:
        ep = os.environ.get('PADDLE_MASTER', '')
        os.environ['MASTER_PORT'] = ep.split(':')[1] if ':' in ep else '29500'
    use_gpu = torch.cuda.is_available() and _default_device().type == 'cuda'
    if backend is None or backend == 'auto':
        # PRA_DIST_BACKEND=gloo rehearses a multi-rank GPU job on ONE device (RCCL refuses two
        # ranks on one GPU): same code paths, host-staged collectives
        backend = os.environ.get('PRA_DIST_BACKEND', 'auto')
    if backend == 'auto':
        backend = 'nccl' if use_gpu else 'gloo'
    if backend in ('rccl', 'xccl', 'bkcl'):
        backend = 'nccl'
    if use_gpu:
        dev_id = _bound_device(env)
        torch.cuda.set_device(dev_id)
        from ..framework.core import set_device
        set_device(f'gpu:{dev_id}')
    to = datetime.timedelta(seconds=timeout_s or int(os.environ.get('PRA_COMM_TIMEOUT', 1800)))
    kw = {}
    if backend == 'nccl' and use_gpu:
        kw['device_id'] = torch.device('cuda', torch.cuda.current_device())
    dist.init_process_group(backend=backend, rank=env.rank, world_size=ws, timeout=to, **kw)
    g = Group(list(range(ws)), None, 0, 'default')
    _default_group[0] = g
    _groups[0] = g
    return g


def _get_default_group():
    if _default_group[0] is None:
        ws = dist.get_world_size() if dist.is_initialized() else 1
        _default_group[0] = Group(list(range(ws)), None, 0, 'default')
        _groups[0] = _default_group[0]
    return _default_group[0]


def get_group(id=0):
    return _groups.get(id, _get_default_group() if id == 0 else None)


def new_group(ranks=None, backend=None, timeout=None):
    ws = dist.get_world_size() if dist.is_initialized() else 1
    ranks = list(range(ws)) if ranks is None else sorted(ranks)
    pg = None
    if dist.is_initialized():
        kw = {}
        if timeout is not None:
            kw['timeout'] = timeout
        pg = dist.new_group(ranks=ranks, backend=backend, **kw)
    gid = _group_counter[0]
    _group_counter[0] += 1
    g = Group(ranks, pg, gid)
    _groups[gid] = g
    return g


def twin_group(group=None):
    """A second communicator over exactly the ranks of ``group`` (its own RCCL stream), so two
    streams of collectives on one rank set (ZeRO-3 parameter all-gathers and gradient
    reduce-scatters) do not serialise behind each other. Collective over the WHOLE job: every
    rank calls it at the same point, each passing its own group; the member lists are
    exchanged and every distinct list is created in one global order (``new_group`` contract)."""
    ws = dist.get_world_size() if dist.is_initialized() else 1
    mine = tuple(range(ws)) if group is None else tuple(sorted(group.ranks))
    if ws == 1:
        return new_group(list(mine))
    lists = [None] * ws
    dist.all_gather_object(lists, mine)
    out = None
    for ranks in sorted(set(tuple(r) for r in lists)):
        g = new_group(list(ranks))
        if ranks == mine:
            out = g
    return out


def destroy_process_group(group=None):
    if group is None:
        if dist.is_initialized():
            dist.destroy_process_group()
        _groups.clear()
        _default_group[0] = None
    elif group.process_group is not None:
        dist.destroy_process_group(group.process_group)


def get_rank(group=None):
    if group is not None:
        return group.rank
    return dist.get_rank() if dist.is_initialized() else 0


def get_world_size(group=None):
    if group is not None:
        return group.nranks
    return dist.get_world_size() if dist.is_initialized() else 1


def get_backend(group=None):
    return dist.get_backend(None if group is None else group.process_group).upper() \
        if dist.is_initialized() else 'UNDEFINED'


def _pg(group):
    return None if group is None else group.process_group


def _single(group):
    return not dist.is_initialized() or (group is not None and group.nranks == 1) or \
        (group is None and dist.get_world_size() == 1)


class _Task:
    def __init__(self, work=None, post=None, name=None):
        self._work, self._post = work, post
        self._wd = None
        if work is not None and _watchdog.enabled():
            self._wd = _watchdog.get_watchdog().track(name or 'collective', work)

    def wait(self):
        if self._work is not None:
            self._work.wait()
            self._work = None
            if self._wd is not None:
                _watchdog.get_watchdog().done(self._wd)
        if self._post is not None:
            self._post()
            self._post = None
        return True

    def is_completed(self):
        return self._work is None or self._work.is_completed()


def _ret(work, sync_op, post=None):
    import sys
    t = _Task(work, post, sys._getframe(1).f_code.co_name)
    if sync_op:
        t.wait()
    return t


def _comm_range(fn):
    """While a profiler records, a collective's host call is a Communication range (the
    profiler's Distributed view; the RCCL kernels themselves come from the device trace)."""
    import functools

    @functools.wraps(fn)
    def wrapper(*a, **k):
        from ..profiler import _hooks
        if not _hooks.ACTIVE:
            return fn(*a, **k)
        from ..profiler import RecordEvent, TracerEventType
        with RecordEvent(fn.__name__, TracerEventType.Communication):
            return fn(*a, **k)
    return wrapper


@_comm_range
def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    if _single(group):
        return _Task()
    return _ret(dist.all_reduce(_u(tensor), _op(op), _pg(group), async_op=True), sync_op)


@_comm_range
def broadcast(tensor, src, group=None, sync_op=True):
    if _single(group):
        return _Task()
    return _ret(dist.broadcast(_u(tensor), src, _pg(group), async_op=True), sync_op)


@_comm_range
def reduce(tensor, dst, op=ReduceOp.SUM, group=None, sync_op=True):
    if _single(group):
        return _Task()
    return _ret(dist.reduce(_u(tensor), dst, _op(op), _pg(group), async_op=True), sync_op)


@_comm_range
def all_gather(tensor_list, tensor, group=None, sync_op=True):
    t = _u(tensor)
    if _single(group):
        if isinstance(tensor_list, list):
            tensor_list.clear()
            tensor_list.append(Tensor(t.clone()))
        return _Task()
    n = get_world_size(group)
    outs = [torch.empty_like(t) for _ in range(n)]
    w = dist.all_gather(outs, t.contiguous(), _pg(group), async_op=True)

    def post():
        tensor_list.clear()
        tensor_list.extend(Tensor(o) for o in outs)
    return _ret(w, sync_op, post)


@_comm_range
def all_gather_into_tensor(out_tensor, in_tensor, group=None, sync_op=True):
    if _single(group):
        _u(out_tensor).copy_(_u(in_tensor).reshape(_u(out_tensor).shape))
        return _Task()
    return _ret(dist.all_gather_into_tensor(_u(out_tensor), _u(in_tensor), _pg(group),
                                            async_op=True), sync_op)


def all_gather_object(object_list, obj, group=None):
    if _single(group):
        object_list.clear()
        object_list.append(obj)
        return
    outs = [None] * get_world_size(group)
    dist.all_gather_object(outs, obj, _pg(group))
    object_list.clear()
    object_list.extend(outs)


def broadcast_object_list(object_list, src=0, group=None):
    if _single(group):
        return
    dist.broadcast_object_list(object_list, src, _pg(group))


def scatter_object_list(out_object_list, in_object_list=None, src=0, group=None):
    if _single(group):
        out_object_list[:] = [in_object_list[0]]
        return
    out = [None]
    dist.scatter_object_list(out, in_object_list, src, _pg(group))
    out_object_list[:] = out


@_comm_range
def reduce_scatter(tensor, tensor_list, op=ReduceOp.SUM, group=None, sync_op=True):
    out = _u(tensor)
    if isinstance(tensor_list, (list, tuple)):
        inp = torch.cat([_u(t).reshape(-1) for t in tensor_list])
    else:
        inp = _u(tensor_list).reshape(-1)
    if _single(group):
        out.copy_(inp.reshape(out.shape))
        return _Task()
    assert out.is_contiguous()
    w = dist.reduce_scatter_tensor(out.view(-1), inp.contiguous(), _op(op), _pg(group),
                                   async_op=True)
    return _ret(w, sync_op)


@_comm_range
def scatter(tensor, tensor_list=None, src=0, group=None, sync_op=True):
    if _single(group):
        if tensor_list:
            _u(tensor).copy_(_u(tensor_list[0]))
        return _Task()
    ins = [_u(t) for t in tensor_list] if (tensor_list and get_rank() == src) else None
    return _ret(dist.scatter(_u(tensor), ins, src, _pg(group), async_op=True), sync_op)


@_comm_range
def alltoall(in_tensor_list, out_tensor_list, group=None, sync_op=True):
    ins = [_u(t).contiguous() for t in in_tensor_list]
    if _single(group):
        out_tensor_list.clear()
        out_tensor_list.extend(Tensor(t.clone()) for t in ins)
        return _Task()
    outs = [torch.empty_like(t) for t in ins]
    if dist.get_backend(_pg(group)) == 'gloo':  # gloo has no alltoall: pairwise p2p exchange
        me = get_rank(group) if group is not None else dist.get_rank()
        ranks = group.ranks if group is not None else list(range(dist.get_world_size()))
        ops = []
        for j, peer in enumerate(ranks):
            if j == me:
                outs[j].copy_(ins[j])
                continue
            ops.append(dist.P2POp(dist.isend, ins[j], peer, _pg(group)))
            ops.append(dist.P2POp(dist.irecv, outs[j], peer, _pg(group)))
        for w_ in dist.batch_isend_irecv(ops):
            w_.wait()
        w = None
    else:
        w = dist.all_to_all(outs, ins, _pg(group), async_op=True)

    def post():
        out_tensor_list.clear()
        out_tensor_list.extend(Tensor(o) for o in outs)
    return _ret(w, sync_op, post)


@_comm_range
def alltoall_single(in_tensor, out_tensor, in_split_sizes=None, out_split_sizes=None, group=None,
                    sync_op=True):
    if _single(group):
        _u(out_tensor).copy_(_u(in_tensor))
        return _Task()
    return _ret(dist.all_to_all_single(_u(out_tensor), _u(in_tensor), out_split_sizes,
                                       in_split_sizes, _pg(group), async_op=True), sync_op)


@_comm_range
def send(tensor, dst=0, group=None, sync_op=True):
    w = dist.isend(_u(tensor).contiguous(), dst, _pg(group))
    return _ret(w, sync_op)


@_comm_range
def recv(tensor, src=0, group=None, sync_op=True):
    w = dist.irecv(_u(tensor), src, _pg(group))
    return _ret(w, sync_op)


@_comm_range
def isend(tensor, dst, group=None):
    return send(tensor, dst, group, False)


@_comm_range
def irecv(tensor, src=None, group=None):
    return recv(tensor, src, group, False)


class P2POp:
    def __init__(self, op, tensor, peer, group=None):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


def batch_isend_irecv(p2p_op_list):
    ops = []
    for p in p2p_op_list:
        fn = dist.isend if p.op in (isend, send, dist.isend) else dist.irecv
        ops.append(dist.P2POp(fn, _u(p.tensor), p.peer, _pg(p.group)))
    return [_Task(w) for w in dist.batch_isend_irecv(ops)]


@_comm_range
def barrier(group=None):
    if _single(group):
        return
    if torch.cuda.is_available() and dist.get_backend(_pg(group)) == 'nccl':
        dist.barrier(_pg(group), device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(_pg(group))


def wait(tensor, group=None, use_calc_stream=True):
    if torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()


def split(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None,
          bias_attr=None, name=None):
    from ..parallel import tensor_parallel as tp
    return tp.split(x, size, operation, axis, num_partitions, gather_out, weight_attr, bias_attr)


class _AllReduceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, pg):
        ctx.pg = pg
        out = t.clone()
        dist.all_reduce(out, group=pg)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        dist.all_reduce(g, group=ctx.pg)
        return g, None


def _all_reduce_autograd(t, group=None):
    return _AllReduceFn.apply(t, _pg(group))


def gloo_init_parallel_env(rank_id, rank_num, server_endpoint):
    os.environ['MASTER_ADDR'], os.environ['MASTER_PORT'] = server_endpoint.split(':')
    os.environ['RANK'], os.environ['WORLD_SIZE'] = str(rank_id), str(rank_num)
    init_parallel_env('gloo')


def gloo_barrier():
    barrier()


def gloo_release():
    pass
