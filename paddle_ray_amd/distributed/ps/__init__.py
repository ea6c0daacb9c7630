"""Parameter-server training: dense and sparse tables on server processes, trainers pull / push.

Parity: the reference's PS mode -- fleet.init(is_collective=False) with a PaddleCloudRoleMaker
reading TRAINING_ROLE / PADDLE_PSERVERS_IP_PORT_LIST / PADDLE_TRAINERS_NUM / PADDLE_TRAINER_ID
(python/paddle/distributed/fleet/base/role_maker.py), fleet.init_server / run_server /
init_worker / stop_worker (fleet/fleet.py), the brpc PS service with dense tables and sparse
(id -> row) tables created on first touch (paddle/fluid/distributed/ps/service/, ps/table/:
memory_dense_table, memory_sparse_table with SGD / Adam rules), and the sparse embedding lookup
that pulls only the rows a batch touches (static.nn.sparse_embedding).

Here the transport is distributed.rpc (TensorPipe): servers are RPC workers ``ps0..psS-1`` and
trainers ``trainer0..trainerT-1`` in one RPC world whose master is the first server endpoint.
Dense tables are placed on server ``crc32(name) % S``; sparse rows on server ``id % S``. Updates
are applied asynchronously on push (the reference's default a_sync mode): SGD or Adam, fp32 on the
server's CPU; trainers keep their compute on the GPU and move only the pulled / pushed rows.
"""
import os
import threading
import zlib

import numpy as np
import torch

from .. import rpc

__all__ = ['PSRole', 'role_from_env', 'init_server', 'run_server', 'init_worker', 'stop_worker',
           'register_dense', 'pull_dense', 'push_dense', 'pull_sparse', 'push_sparse', 'SparseEmbedding',
           'DistributedOptimizer']


class PSRole:
    def __init__(self, role, index, n_servers, n_trainers, server_endpoints):
        self.role, self.index = role, index
        self.n_servers, self.n_trainers = n_servers, n_trainers
        self.server_endpoints = server_endpoints

    @property
    def is_server(self):
        return self.role == 'PSERVER'

    @property
    def rpc_rank(self):
        return self.index if self.is_server else self.n_servers + self.index

    @property
    def name(self):
        return f'ps{self.index}' if self.is_server else f'trainer{self.index}'


def role_from_env():
    """The reference PaddleCloudRoleMaker's environment contract."""
    role = os.environ.get('TRAINING_ROLE', 'TRAINER').upper()
    eps = [e for e in os.environ['PADDLE_PSERVERS_IP_PORT_LIST'].split(',') if e]
    n_tr = int(os.environ['PADDLE_TRAINERS_NUM'])
    if role == 'PSERVER':
        cur = os.environ.get('PADDLE_PSERVER_ID')
        if cur is not None:
            idx = int(cur)
        else:
            ep = '%s:%s' % (os.environ['POD_IP'], os.environ['PADDLE_PORT'])
            idx = eps.index(ep)
    else:
        idx = int(os.environ['PADDLE_TRAINER_ID'])
    return PSRole(role, idx, len(eps), n_tr, eps)


_ROLE = [None]


def _init(role):
    _ROLE[0] = role
    os.environ.setdefault('PADDLE_WORKER_ENDPOINT', role.server_endpoints[role.index] if role.is_server
                          else '127.0.0.1:0')
    rpc.init_rpc(role.name, rank=role.rpc_rank, world_size=role.n_servers + role.n_trainers,
                 master_endpoint=role.server_endpoints[0])


def init_server(role=None):
    _init(role or role_from_env())


def run_server():
    """Serve until every trainer called stop_worker (rpc shutdown is collective)."""
    rpc.shutdown()


def init_worker(role=None):
    _init(role or role_from_env())


def stop_worker():
    rpc.shutdown()


# ----------------------------------------------------------------------------- server side
class _Rule:
    """Per-table update rule (ps/table sgd / adam accessors)."""

    def __init__(self, kind='sgd', lr=0.01, beta1=0.9, beta2=0.999, eps=1e-8):
        self.kind, self.lr, self.b1, self.b2, self.eps = kind, lr, beta1, beta2, eps

    def state(self, shape):
        return {} if self.kind == 'sgd' else {'m': np.zeros(shape, np.float32), 'v': np.zeros(shape, np.float32),
                                              't': 0}

    def apply(self, w, g, st):
        if self.kind == 'sgd':
            w -= self.lr * g
            return
        st['t'] += 1
        st['m'] *= self.b1
        st['m'] += (1 - self.b1) * g
        st['v'] *= self.b2
        st['v'] += (1 - self.b2) * g * g
        mh = st['m'] / (1 - self.b1 ** st['t'])
        vh = st['v'] / (1 - self.b2 ** st['t'])
        w -= self.lr * mh / (np.sqrt(vh) + self.eps)


_LOCK = threading.Lock()
_DENSE = {}    # name -> [w, rule, state]
_SPARSE = {}   # name -> {'dim', 'rule', 'init', 'rows': {id: [row, state]}, 'seed'}


def _srv_create_dense(name, value, rule):
    with _LOCK:
        if name not in _DENSE:   # first trainer's initial value wins
            w = np.array(value, dtype=np.float32, copy=True)
            _DENSE[name] = [w, _Rule(**rule), _Rule(**rule).state(w.shape)]


def _srv_pull_dense(names):
    with _LOCK:
        return [_DENSE[n][0].copy() for n in names]


def _srv_push_dense(grads):
    with _LOCK:
        for n, g in grads.items():
            w, rule, st = _DENSE[n]
            rule.apply(w, np.asarray(g, np.float32), st)


def _srv_create_sparse(name, dim, rule, init_std, seed):
    with _LOCK:
        if name not in _SPARSE:
            _SPARSE[name] = {'dim': dim, 'rule': _Rule(**rule), 'std': init_std, 'seed': seed, 'rows': {}}


def _row(tab, i):
    r = tab['rows'].get(i)
    if r is None:   # created on first touch, deterministically from (seed, id)
        g = np.random.default_rng([tab['seed'], int(i)])
        w = (g.standard_normal(tab['dim']) * tab['std']).astype(np.float32)
        r = tab['rows'][i] = [w, tab['rule'].state((tab['dim'],))]
    return r


def _srv_pull_sparse(name, ids):
    with _LOCK:
        tab = _SPARSE[name]
        return np.stack([_row(tab, i)[0] for i in ids]) if len(ids) else np.zeros((0, tab['dim']), np.float32)


def _srv_push_sparse(name, ids, grads):
    with _LOCK:
        tab = _SPARSE[name]
        for i, g in zip(ids, np.asarray(grads, np.float32)):
            w, st = _row(tab, i)
            tab['rule'].apply(w, g, st)


def _srv_sparse_size(name):
    with _LOCK:
        return len(_SPARSE[name]['rows'])


# ----------------------------------------------------------------------------- trainer side
def _servers():
    return _ROLE[0].n_servers


def _dense_server(name):
    return 'ps%d' % (zlib.crc32(name.encode()) % _servers())


def register_dense(name, value, optimizer='sgd', lr=0.01, **kw):
    rule = dict(kind=optimizer, lr=lr, **kw)
    rpc.rpc_sync(_dense_server(name), _srv_create_dense,
                 args=(name, value.detach().float().cpu().numpy(), rule))


def pull_dense(names):
    by = {}
    for n in names:
        by.setdefault(_dense_server(n), []).append(n)
    futs = {s: rpc.rpc_async(s, _srv_pull_dense, args=(ns,)) for s, ns in by.items()}
    out = {}
    for s, ns in by.items():
        for n, v in zip(ns, futs[s].wait()):
            out[n] = torch.from_numpy(v)
    return [out[n] for n in names]


def push_dense(grads):
    by = {}
    for n, g in grads.items():
        by.setdefault(_dense_server(n), {})[n] = g.detach().float().cpu().numpy()
    for f in [rpc.rpc_async(s, _srv_push_dense, args=(gs,)) for s, gs in by.items()]:
        f.wait()


def create_sparse_table(name, dim, optimizer='sgd', lr=0.01, init_std=0.01, seed=0, **kw):
    rule = dict(kind=optimizer, lr=lr, **kw)
    for s in range(_servers()):
        rpc.rpc_sync('ps%d' % s, _srv_create_sparse, args=(name, dim, rule, init_std, seed))


def _split_ids(ids):
    S = _servers()
    parts = {}
    for pos, i in enumerate(ids):
        parts.setdefault(int(i) % S, ([], []))
        parts[int(i) % S][0].append(int(i))
        parts[int(i) % S][1].append(pos)
    return parts


def pull_sparse(name, ids):
    """Rows [len(ids), dim] (fp32, CPU) of sparse table ``name``."""
    ids = [int(i) for i in ids]
    parts = _split_ids(ids)
    futs = {s: rpc.rpc_async('ps%d' % s, _srv_pull_sparse, args=(name, p[0])) for s, p in parts.items()}
    out = None
    for s, (sid, pos) in parts.items():
        rows = futs[s].wait()
        if out is None:
            out = np.zeros((len(ids), rows.shape[1]), np.float32)
        out[pos] = rows
    return torch.from_numpy(out if out is not None else np.zeros((0, 0), np.float32))


def push_sparse(name, ids, grads):
    ids = [int(i) for i in ids]
    g = grads.detach().float().cpu().numpy()
    parts = _split_ids(ids)
    for f in [rpc.rpc_async('ps%d' % s, _srv_push_sparse, args=(name, sid, g[pos])) for s, (sid, pos)
              in parts.items()]:
        f.wait()


def sparse_table_size(name):
    return sum(rpc.rpc_sync('ps%d' % s, _srv_sparse_size, args=(name,)) for s in range(_servers()))


class SparseEmbedding(torch.nn.Module):
    """Embedding whose table lives on the servers: forward pulls the batch's unique rows, the
    backward pushes their gradients (static.nn.sparse_embedding / distributed lookup table)."""

    def __init__(self, name, dim, optimizer='sgd', lr=0.01, init_std=0.01, seed=0, **kw):
        super().__init__()
        self.table, self.dim = name, dim
        create_sparse_table(name, dim, optimizer, lr, init_std, seed, **kw)

    def forward(self, ids):
        flat = ids.reshape(-1)
        if flat.numel() == 0:
            return torch.zeros(*ids.shape, self.dim, device=ids.device)
        uniq, inv = torch.unique(flat.cpu(), return_inverse=True)
        rows = pull_sparse(self.table, uniq.tolist()).to(ids.device).requires_grad_()
        table, uid = self.table, uniq.tolist()
        rows.register_hook(lambda g: push_sparse(table, uid, g))
        return rows[inv.to(ids.device)].reshape(*ids.shape, self.dim)


class DistributedOptimizer:
    """Dense parameters trained on the servers: ``step()`` pushes the gradients and pulls the
    updated values back into the parameters (async PS mode); ``clear_grad()`` as usual."""

    def __init__(self, params, optimizer='sgd', lr=0.01, prefix='dense', **kw):
        self.params = [p for p in params]
        self.names = ['%s.%d' % (prefix, i) for i in range(len(self.params))]
        for n, p in zip(self.names, self.params):
            register_dense(n, p.data, optimizer, lr, **kw)
        self._pull()

    def _pull(self):
        with torch.no_grad():
            for p, v in zip(self.params, pull_dense(self.names)):
                p.copy_(v.to(p.device, p.dtype))

    def step(self):
        push_dense({n: p.grad for n, p in zip(self.names, self.params) if p.grad is not None})
        self._pull()

    def clear_grad(self):
        for p in self.params:
            p.grad = None

    zero_grad = clear_grad
