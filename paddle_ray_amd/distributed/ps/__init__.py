"""Parameter-server training: dense and sparse tables on server processes, trainers pull / push.

Parity: the reference's PS mode -- fleet.init(is_collective=False) with a PaddleCloudRoleMaker
reading TRAINING_ROLE / PADDLE_PSERVERS_IP_PORT_LIST / PADDLE_TRAINERS_NUM / PADDLE_TRAINER_ID
(python/paddle/distributed/fleet/base/role_maker.py), fleet.init_server(dirname) / run_server /
init_worker / stop_worker / save_persistables (fleet/fleet.py:695,934; the_one_ps.py:1340
`_init_server`, :1459 `_save_sparse_params`, :1644 `_load_sparse_params`, :1730
`_save_persistables`), the brpc PS service with dense tables and sparse (id -> row) tables
created on first touch (paddle/fluid/distributed/ps/table: memory_dense_table,
memory_sparse_table with SGD / Adam rules), async (a_sync) and sync update modes, and the sparse
embedding lookup that pulls only the rows a batch touches (static.nn.sparse_embedding).

Design (this framework's own):
* transport = distributed.rpc (TensorPipe): servers are RPC workers ``ps0..psS-1`` and trainers
  ``trainer0..trainerT-1`` in one RPC world whose master is the first server endpoint;
* a dense table lives on server ``crc32(name) % S``; sparse row ``id`` on server ``id % S``;
* every table has its own lock -- pushes to different tables never serialise on each other;
* sparse tables are contiguous arrays (rows, and Adam moments / per-row step counts) with an
  id -> slot index; a push updates all its rows with one vectorised rule application;
* ``async`` (strategy.a_sync = True, the default): a push is applied on arrival;
  ``sync`` (a_sync = False): a table accumulates the pushes of one step from every trainer and
  applies their MEAN once all T arrived (= serial SGD on the union of the trainers' batches),
  then bumps its version; a pull names the version it needs and waits for it;
* persistence: ``save(dirname)`` has every server write the tables it holds (dense
  ``dense/<name>.npz``, sparse ``sparse/<name>/part-<server>-of-<S>.npz``, parameters plus the
  optimizer state unless mode 2 = base); ``init_server(dirname)`` preloads them -- dense tables
  by their owner, sparse shards re-partitioned by ``id % S`` (any server count) -- and a
  trainer's table creation then takes the loaded values instead of its initial ones.
"""
import glob
import json
import os
import threading
import zlib

import numpy as np
import torch

from .. import rpc

__all__ = ['PSRole', 'role_from_env', 'init_server', 'run_server', 'init_worker', 'stop_worker',
           'register_dense', 'pull_dense', 'push_dense', 'pull_sparse', 'push_sparse', 'SparseEmbedding',
           'DistributedOptimizer', 'set_mode', 'get_mode', 'save', 'load', 'sparse_table_size']

_WAIT_S = 600.0   # a sync-mode pull waits at most this long for the other trainers' pushes


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
_MODE = ['async']


def set_mode(mode):
    """'async' (strategy.a_sync = True) or 'sync'; tables created afterwards use it."""
    if mode not in ('async', 'sync'):
        raise ValueError(f"PS mode must be 'async' or 'sync', got {mode!r}")
    _MODE[0] = mode


def get_mode():
    return _MODE[0]


def _init(role):
    _ROLE[0] = role
    os.environ.setdefault('PADDLE_WORKER_ENDPOINT', role.server_endpoints[role.index] if role.is_server
                          else '127.0.0.1:0')
    rpc.init_rpc(role.name, rank=role.rpc_rank, world_size=role.n_servers + role.n_trainers,
                 master_endpoint=role.server_endpoints[0])


def init_server(role=None, dirname=None):
    """Join the RPC world as a server; with ``dirname`` preload the tables a previous ``save``
    wrote (this server's dense tables and its share of every sparse table)."""
    role = role or role_from_env()
    if dirname:
        _load_dir(dirname, role.index, role.n_servers)
    _init(role)


def run_server():
    """Serve until every trainer called stop_worker (rpc shutdown is collective)."""
    rpc.shutdown()


def init_worker(role=None):
    _init(role or role_from_env())


def stop_worker():
    rpc.shutdown()


# ----------------------------------------------------------------------------- server side
def _n_trainers():
    r = _ROLE[0]
    return r.n_trainers if r is not None else 1


class _Rule:
    """Update rule of a table (ps/table sgd / adam accessors), vectorised over rows."""

    def __init__(self, kind='sgd', lr=0.01, beta1=0.9, beta2=0.999, eps=1e-8):
        if kind not in ('sgd', 'adam'):
            raise ValueError(f"PS table optimizer must be 'sgd' or 'adam', got {kind!r}")
        self.kind, self.lr, self.b1, self.b2, self.eps = kind, lr, beta1, beta2, eps

    def config(self):
        return {'kind': self.kind, 'lr': self.lr, 'beta1': self.b1, 'beta2': self.b2, 'eps': self.eps}

    def apply(self, w, g, m=None, v=None, t=None):
        """w -= update(g) in place; m / v / t (Adam moments and step count: a scalar for a dense
        table, one per row for sparse rows) are updated in place and the new t returned."""
        if self.kind == 'sgd':
            w -= self.lr * g
            return t
        t = t + 1
        m *= self.b1
        m += (1 - self.b1) * g
        v *= self.b2
        v += (1 - self.b2) * g * g
        tt = t if np.ndim(t) == 0 else np.asarray(t, np.float64).reshape((-1,) + (1,) * (g.ndim - 1))
        mh = m / (1 - self.b1 ** tt)
        vh = v / (1 - self.b2 ** tt)
        w -= (self.lr * mh / (np.sqrt(vh) + self.eps)).astype(np.float32)
        return t


class _DenseTable:
    def __init__(self, w, rule, mode, state=None):
        self.w = w
        self.rule = rule
        self.mode = mode
        self.m = np.zeros_like(w) if rule.kind == 'adam' else None
        self.v = np.zeros_like(w) if rule.kind == 'adam' else None
        self.t = 0
        if state:
            self.m, self.v, self.t = state.get('m', self.m), state.get('v', self.v), int(state.get('t', 0))
        self.version = 0
        self.pending, self.count = None, 0
        self.cond = threading.Condition()

    def push(self, g):
        g = np.asarray(g, np.float32).reshape(self.w.shape)
        with self.cond:
            if self.mode == 'async':
                self.t = self.rule.apply(self.w, g, self.m, self.v, self.t)
                self.version += 1
                return
            self.pending = g.copy() if self.pending is None else self.pending + g
            self.count += 1
            if self.count >= _n_trainers():
                self.t = self.rule.apply(self.w, self.pending / self.count, self.m, self.v, self.t)
                self.pending, self.count = None, 0
                self.version += 1
                self.cond.notify_all()

    def pull(self, min_version=0):
        with self.cond:
            if not self.cond.wait_for(lambda: self.version >= min_version, timeout=_WAIT_S):
                raise TimeoutError(f"PS sync pull: version {min_version} not reached ({self.version})")
            return self.w.copy()


class _SparseTable:
    def __init__(self, dim, rule, std, seed, mode):
        self.dim, self.rule, self.std, self.seed, self.mode = dim, rule, std, seed, mode
        self.index = {}
        self.n = 0
        cap = 1024
        self.ids = np.zeros(cap, np.int64)
        self.W = np.zeros((cap, dim), np.float32)
        adam = rule.kind == 'adam'
        self.M = np.zeros((cap, dim), np.float32) if adam else None
        self.V = np.zeros((cap, dim), np.float32) if adam else None
        self.T = np.zeros(cap, np.int64) if adam else None
        self.version = 0
        self.pending, self.count = [], 0
        self.cond = threading.Condition()

    def _grow(self, need):
        cap = self.W.shape[0]
        if need <= cap:
            return
        new = max(need, 2 * cap)
        self.ids = np.resize(self.ids, new)
        W = np.zeros((new, self.dim), np.float32)
        W[:self.n] = self.W[:self.n]
        self.W = W
        if self.M is not None:
            for name in ('M', 'V'):
                a = np.zeros((new, self.dim), np.float32)
                a[:self.n] = getattr(self, name)[:self.n]
                setattr(self, name, a)
            T = np.zeros(new, np.int64)
            T[:self.n] = self.T[:self.n]
            self.T = T

    def _init_row(self, i):
        # deterministic from (seed, id): the same row whichever server / trainer touches it first
        g = np.random.default_rng([self.seed, int(i)])
        return (g.standard_normal(self.dim) * self.std).astype(np.float32)

    def slots(self, ids):
        """Row slots of ``ids`` (rows created on first touch)."""
        idx = self.index
        out = np.fromiter((idx.get(int(i), -1) for i in ids), np.int64, count=len(ids))
        miss = np.nonzero(out < 0)[0]
        if len(miss):
            new_ids = []
            for k in miss:
                i = int(ids[k])
                s = idx.get(i)
                if s is None:
                    s = idx[i] = self.n + len(new_ids)
                    new_ids.append(i)
                out[k] = s
            self._grow(self.n + len(new_ids))
            for j, i in enumerate(new_ids):
                self.ids[self.n + j] = i
                self.W[self.n + j] = self._init_row(i)
            self.n += len(new_ids)
        return out

    def load_rows(self, ids, W, M=None, V=None, T=None):
        s = self.slots(ids)
        self.W[s] = W
        if self.M is not None and M is not None:
            self.M[s], self.V[s], self.T[s] = M, V, T

    def _apply(self, ids, grads):
        s = self.slots(ids)
        if self.rule.kind == 'sgd':
            self.W[s] -= self.rule.lr * grads
            return
        W, M, V = self.W[s], self.M[s], self.V[s]
        T = self.rule.apply(W, grads, M, V, self.T[s])
        self.W[s], self.M[s], self.V[s], self.T[s] = W, M, V, T

    def push(self, ids, grads):
        ids = np.asarray(ids, np.int64).reshape(-1)
        grads = np.asarray(grads, np.float32).reshape(len(ids), self.dim)
        with self.cond:
            if self.mode == 'async':
                if len(ids):
                    uid, inv = np.unique(ids, return_inverse=True)
                    if len(uid) != len(ids):   # duplicate ids in one push: their gradients add
                        acc = np.zeros((len(uid), self.dim), np.float32)
                        np.add.at(acc, inv, grads)
                        ids, grads = uid, acc
                    self._apply(ids, grads)
                self.version += 1
                return
            self.pending.append((ids, grads))
            self.count += 1
            if self.count >= _n_trainers():
                all_ids = np.concatenate([i for i, _ in self.pending])
                if len(all_ids):
                    all_g = np.concatenate([g for _, g in self.pending])
                    uid, inv = np.unique(all_ids, return_inverse=True)
                    acc = np.zeros((len(uid), self.dim), np.float32)
                    np.add.at(acc, inv, all_g)
                    self._apply(uid, acc / self.count)
                self.pending, self.count = [], 0
                self.version += 1
                self.cond.notify_all()

    def pull(self, ids, min_version=0):
        ids = np.asarray(ids, np.int64).reshape(-1)
        with self.cond:
            if not self.cond.wait_for(lambda: self.version >= min_version, timeout=_WAIT_S):
                raise TimeoutError(f"PS sync pull: version {min_version} not reached ({self.version})")
            if not len(ids):
                return np.zeros((0, self.dim), np.float32)
            return self.W[self.slots(ids)].copy()


_TABLES_LOCK = threading.Lock()   # guards the table dicts only (creation / lookup)
_DENSE = {}
_SPARSE = {}
_PRELOAD = {'dense': {}, 'sparse': {}}


def _srv_create_dense(name, value, rule, mode='async'):
    with _TABLES_LOCK:
        if name in _DENSE:        # first trainer's creation wins
            return
        pre = _PRELOAD['dense'].pop(name, None)
        r = _Rule(**rule)
        if pre is not None:
            _DENSE[name] = _DenseTable(pre['w'], r, mode, pre)
        else:
            _DENSE[name] = _DenseTable(np.array(value, dtype=np.float32, copy=True), r, mode)


def _srv_pull_dense(names, min_version=0):
    return [_DENSE[n].pull(min_version) for n in names]


def _srv_push_dense(grads):
    for n, g in grads.items():
        _DENSE[n].push(g)


def _srv_create_sparse(name, dim, rule, init_std, seed, mode='async'):
    with _TABLES_LOCK:
        if name in _SPARSE:
            return
        tab = _SPARSE[name] = _SparseTable(dim, _Rule(**rule), init_std, seed, mode)
        pre = _PRELOAD['sparse'].pop(name, None)
        if pre is not None and len(pre['ids']):
            tab.load_rows(pre['ids'], pre['W'], pre.get('M'), pre.get('V'), pre.get('T'))


def _srv_pull_sparse(name, ids, min_version=0):
    return _SPARSE[name].pull(ids, min_version)


def _srv_push_sparse(name, ids, grads):
    _SPARSE[name].push(ids, grads)


def _srv_sparse_size(name):
    tab = _SPARSE[name]
    with tab.cond:
        return tab.n


def _srv_save(dirname, mode, server, n_servers, table=None):
    """Write this server's tables (mode 0 / 1: parameters + optimizer state, 2: parameters)."""
    full = mode != 2
    os.makedirs(os.path.join(dirname, 'dense'), exist_ok=True)
    with _TABLES_LOCK:
        dense = {k: v for k, v in _DENSE.items() if table is None or k == table}
        sparse = {k: v for k, v in _SPARSE.items() if table is None or k == table}
    for name, t in dense.items():
        with t.cond:
            arrs = {'w': t.w.copy()}
            if full and t.m is not None:
                arrs.update(m=t.m.copy(), v=t.v.copy(), t=np.array(t.t))
            meta = {'rule': t.rule.config(), 'version': t.version}
        np.savez(os.path.join(dirname, 'dense', f'{name}.npz'), meta=np.array(json.dumps(meta)), **arrs)
    for name, t in sparse.items():
        d = os.path.join(dirname, 'sparse', name)
        os.makedirs(d, exist_ok=True)
        with t.cond:
            n = t.n
            arrs = {'ids': t.ids[:n].copy(), 'W': t.W[:n].copy()}
            if full and t.M is not None:
                arrs.update(M=t.M[:n].copy(), V=t.V[:n].copy(), T=t.T[:n].copy())
            meta = {'dim': t.dim, 'rule': t.rule.config(), 'std': t.std, 'seed': t.seed}
        np.savez(os.path.join(d, f'part-{server}-of-{n_servers}.npz'), meta=np.array(json.dumps(meta)), **arrs)
    return {'dense': sorted(dense), 'sparse': {k: int(v.n) for k, v in sparse.items()}}


def _load_dir(dirname, server, n_servers):
    """Preload what ``save`` wrote: the dense tables this server owns and every sparse row
    with id % n_servers == server."""
    for f in sorted(glob.glob(os.path.join(dirname, 'dense', '*.npz'))):
        name = os.path.basename(f)[:-4]
        if zlib.crc32(name.encode()) % n_servers != server:
            continue
        with np.load(f, allow_pickle=False) as z:
            d = {k: z[k] for k in z.files if k != 'meta'}
        if 't' in d:
            d['t'] = int(d['t'])
        _PRELOAD['dense'][name] = d
    for tdir in sorted(glob.glob(os.path.join(dirname, 'sparse', '*'))):
        name = os.path.basename(tdir)
        parts = {}
        for f in sorted(glob.glob(os.path.join(tdir, 'part-*.npz'))):
            with np.load(f, allow_pickle=False) as z:
                keep = (z['ids'] % n_servers) == server
                for k in z.files:
                    if k != 'meta':
                        parts.setdefault(k, []).append(z[k][keep])
        if parts:
            _PRELOAD['sparse'][name] = {k: np.concatenate(v) for k, v in parts.items()}


def _srv_load(dirname, server, n_servers, table=None):
    """Load saved tables into this running server: existing tables take the saved values (and
    optimizer state), tables not created yet are preloaded for their creation."""
    _load_dir(dirname, server, n_servers)
    loaded = []
    with _TABLES_LOCK:
        for name in list(_PRELOAD['dense']):
            if (table is None or name == table) and name in _DENSE:
                pre = _PRELOAD['dense'].pop(name)
                t = _DENSE[name]
                with t.cond:
                    t.w[...] = pre['w']
                    if t.m is not None and 'm' in pre:
                        t.m[...], t.v[...], t.t = pre['m'], pre['v'], int(pre['t'])
                loaded.append(name)
        for name in list(_PRELOAD['sparse']):
            if (table is None or name == table) and name in _SPARSE:
                pre = _PRELOAD['sparse'].pop(name)
                t = _SPARSE[name]
                with t.cond:
                    if len(pre['ids']):
                        t.load_rows(pre['ids'], pre['W'], pre.get('M'), pre.get('V'), pre.get('T'))
                loaded.append(name)
    return loaded


# ----------------------------------------------------------------------------- trainer side
def _servers():
    return _ROLE[0].n_servers


def _dense_server(name):
    return 'ps%d' % (zlib.crc32(name.encode()) % _servers())


def register_dense(name, value, optimizer='sgd', lr=0.01, mode=None, **kw):
    rule = dict(kind=optimizer, lr=lr, **kw)
    rpc.rpc_sync(_dense_server(name), _srv_create_dense,
                 args=(name, value.detach().float().cpu().numpy(), rule, mode or _MODE[0]))


def pull_dense(names, min_version=0):
    by = {}
    for n in names:
        by.setdefault(_dense_server(n), []).append(n)
    futs = {s: rpc.rpc_async(s, _srv_pull_dense, args=(ns, min_version)) for s, ns in by.items()}
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


def create_sparse_table(name, dim, optimizer='sgd', lr=0.01, init_std=0.01, seed=0, mode=None, **kw):
    rule = dict(kind=optimizer, lr=lr, **kw)
    for s in range(_servers()):
        rpc.rpc_sync('ps%d' % s, _srv_create_sparse, args=(name, dim, rule, init_std, seed, mode or _MODE[0]))


def _split_ids(ids):
    """{server: (ids array, positions array)} for an int64 id array (vectorised)."""
    S = _servers()
    owner = ids % S
    out = {}
    for s in np.unique(owner):
        pos = np.nonzero(owner == s)[0]
        out[int(s)] = (ids[pos], pos)
    return out


def pull_sparse(name, ids, min_version=0, dim=None, all_servers=False):
    """Rows [len(ids), dim] (fp32, CPU) of sparse table ``name``. ``all_servers``: ask every
    server (a sync-mode pull must wait on each server's table version)."""
    ids = np.asarray(ids, np.int64).reshape(-1)
    parts = _split_ids(ids)
    if all_servers:
        for s in range(_servers()):
            parts.setdefault(s, (ids[:0], np.zeros(0, np.int64)))
    futs = {s: rpc.rpc_async('ps%d' % s, _srv_pull_sparse, args=(name, p[0], min_version)) for s, p in parts.items()}
    out = None
    for s, (sid, pos) in parts.items():
        rows = futs[s].wait()
        if out is None:
            out = np.zeros((len(ids), rows.shape[1]), np.float32)
        if len(pos):
            out[pos] = rows
    if out is None:
        out = np.zeros((0, dim or 0), np.float32)
    return torch.from_numpy(out)


def push_sparse(name, ids, grads, all_servers=False):
    """Push row gradients; ``all_servers``: every server receives a (possibly empty) push, as a
    sync-mode step needs one push per trainer on each server."""
    ids = np.asarray(ids, np.int64).reshape(-1)
    g = grads.detach().float().cpu().numpy().reshape(len(ids), -1)
    parts = _split_ids(ids)
    if all_servers:
        for s in range(_servers()):
            parts.setdefault(s, (ids[:0], np.zeros(0, np.int64)))
    for f in [rpc.rpc_async('ps%d' % s, _srv_push_sparse, args=(name, sid, g[pos])) for s, (sid, pos)
              in parts.items()]:
        f.wait()


def sparse_table_size(name):
    return sum(rpc.rpc_sync('ps%d' % s, _srv_sparse_size, args=(name,)) for s in range(_servers()))


def save(dirname, mode=0, table=None):
    """Every server writes the tables it holds under ``dirname`` (call from one trainer, e.g.
    fleet.save_persistables on the first worker); ``table``: only that one. Returns the servers'
    table inventories."""
    S = _servers()
    futs = [rpc.rpc_async('ps%d' % s, _srv_save, args=(dirname, mode, s, S, table)) for s in range(S)]
    return [f.wait() for f in futs]


def load(dirname, table=None):
    """Running servers load what ``save`` wrote (fleet.load_model / load_one_table)."""
    S = _servers()
    futs = [rpc.rpc_async('ps%d' % s, _srv_load, args=(dirname, s, S, table)) for s in range(S)]
    return [f.wait() for f in futs]


class SparseEmbedding(torch.nn.Module):
    """Embedding whose table lives on the servers: forward pulls the batch's unique rows, the
    backward pushes their gradients (static.nn.sparse_embedding / distributed lookup table).
    Ids on the host (the usual reader output) are used as they are; device ids are copied to
    the host once, since the pull itself is a host RPC. In sync mode every forward/backward is
    one step: the pull waits for the previous step's merged update on every server."""

    def __init__(self, name, dim, optimizer='sgd', lr=0.01, init_std=0.01, seed=0, mode=None, **kw):
        super().__init__()
        self.table, self.dim = name, dim
        self.mode = mode or _MODE[0]
        self._steps = 0
        create_sparse_table(name, dim, optimizer, lr, init_std, seed, mode=self.mode, **kw)

    def forward(self, ids):
        sync = self.mode == 'sync'
        host = ids.detach().reshape(-1)
        host = host.numpy() if host.device.type == 'cpu' else host.cpu().numpy()
        uniq, inv = np.unique(host.astype(np.int64), return_inverse=True)
        rows = pull_sparse(self.table, uniq, self._steps if sync else 0, self.dim, all_servers=sync)
        rows = rows.to(ids.device).requires_grad_()
        table = self.table

        def hook(g, _u=uniq):
            push_sparse(table, _u, g, all_servers=sync)
        rows.register_hook(hook)
        self._steps += 1
        inv_t = torch.from_numpy(inv.astype(np.int64)).to(ids.device)
        return rows[inv_t].reshape(*ids.shape, self.dim)


class DistributedOptimizer:
    """Dense parameters trained on the servers: ``step()`` pushes the gradients and pulls the
    updated values back into the parameters; in sync mode the pull waits until every trainer's
    push of this step was merged (a parameter without a gradient pushes zeros)."""

    def __init__(self, params, optimizer='sgd', lr=0.01, prefix='dense', mode=None, **kw):
        self.params = [p for p in params]
        self.names = ['%s.%d' % (prefix, i) for i in range(len(self.params))]
        self.mode = mode or _MODE[0]
        self._version = 0
        for n, p in zip(self.names, self.params):
            register_dense(n, p.data, optimizer, lr, mode=self.mode, **kw)
        self._pull(0)

    def _pull(self, min_version):
        with torch.no_grad():
            for p, v in zip(self.params, pull_dense(self.names, min_version)):
                p.copy_(v.to(p.device, p.dtype))

    def step(self):
        if self.mode == 'sync':
            push_dense({n: (p.grad if p.grad is not None else torch.zeros_like(p))
                        for n, p in zip(self.names, self.params)})
            self._version += 1
            self._pull(self._version)
        else:
            push_dense({n: p.grad for n, p in zip(self.names, self.params) if p.grad is not None})
            self._pull(0)

    def clear_grad(self):
        for p in self.params:
            p.grad = None

    zero_grad = clear_grad
