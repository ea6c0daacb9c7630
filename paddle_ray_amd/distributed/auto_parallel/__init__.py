"""Semi-automatic parallelism: process meshes, sharding annotations, reshard and a training Engine.

Parity: reference python/paddle/distributed/auto_parallel/__init__.py (Strategy, ProcessMesh,
Engine, shard_tensor, shard_op, recompute, fetch), process_mesh.py:45 (ProcessMesh),
interface.py:28 (shard_tensor: `shard_spec[i]` names the mesh dim tensor dim i is split over),
engine.py (Engine.fit/evaluate/predict/save/load), strategy.py (Strategy sections), reshard.py.

MI355X-native design: the reference annotates a static program, then runs completion +
partitioner + reshard passes to emit per-rank programs. Here annotation is eager and physical:
`shard_tensor` attaches a `DistAttr` (mesh + dims_mapping) and keeps only the local shard on the
rank (one process per GPU; a 1.3B model's shards fit the 288 GB HBM of one MI355X many times over,
so there is no reason to defer placement to a compiler). `reshard` is one all_gather per sharded
mesh axis (RCCL over xGMI; the gather is autograd-aware, its backward is the local slice) followed
by a local slice. The Engine data-parallelises over mesh axis 0 (the batch axis, as in the
reference's default DP completion) and all-reduces each gradient over the mesh axes its
parameter is replicated on, so tensor-parallel (sharded) parameters sync only over DP.

Static programs take the reference's route: in static mode `shard_tensor` only annotates, and
`parallelize(program)` runs completion + partitioning + reshard (static_passes.py) to produce this
rank's program with local parameter shards and the collectives the placements imply.
"""
import copy
import os

import numpy as np
import torch

from ...framework.core import Tensor, Parameter, _u
from .. import collective as C

__all__ = ['ProcessMesh', 'DistAttr', 'Strategy', 'Engine', 'shard_tensor', 'shard_op', 'reshard',
           'recompute', 'fetch', 'get_current_process_mesh', 'dist_attr']

_mesh_stack = []
_axis_groups = {}
_fetches = {}


# ============================================================================================
# ProcessMesh
# ============================================================================================
class ProcessMesh:
    """N-d arrangement of ranks with named dims (reference process_mesh.py:45).

    `with mesh:` makes it the default mesh of shard_tensor/shard_op inside the block."""

    def __init__(self, mesh=None, dim_names=None, shape=None, process_ids=None):
        if mesh is None:
            assert shape is not None and process_ids is not None, "give mesh or (shape, process_ids)"
            mesh = np.array(process_ids).reshape(shape)
        self._mesh = np.array(mesh, dtype=np.int64)
        if self._mesh.ndim == 0:
            self._mesh = self._mesh.reshape(1)
        assert len(np.unique(self._mesh)) == self._mesh.size, "process ids in a mesh must be unique"
        if dim_names is None:
            dim_names = [f"d{i}" for i in range(self._mesh.ndim)]
        assert len(dim_names) == self._mesh.ndim, "one name per mesh dim"
        assert len(set(dim_names)) == len(dim_names), "mesh dim names must be unique"
        self._dim_names = list(dim_names)

    mesh = property(lambda self: self._mesh)
    shape = property(lambda self: list(self._mesh.shape))
    ndim = property(lambda self: self._mesh.ndim)
    dim_names = property(lambda self: list(self._dim_names))
    process_ids = property(lambda self: [int(x) for x in self._mesh.flatten()])
    processes = process_ids

    def get_dim_size(self, dim):
        return self._mesh.shape[self._dim(dim)]

    def _dim(self, dim):
        return self._dim_names.index(dim) if isinstance(dim, str) else int(dim)

    def contains(self, rank):
        return int(rank) in self.process_ids

    def coord(self, rank=None):
        """Mesh coordinate of `rank` (default: this process), None when outside the mesh."""
        rank = C.get_rank() if rank is None else rank
        hit = np.argwhere(self._mesh == rank)
        return None if len(hit) == 0 else [int(v) for v in hit[0]]

    def __getitem__(self, index):
        if isinstance(index, str):  # slice along a named dim keeps that dim only for this coord
            raise TypeError("index a ProcessMesh with ints/slices")
        sub = self._mesh[index]
        if not isinstance(index, tuple):
            index = (index,)
        names = [n for i, n in enumerate(self._dim_names)
                 if i >= len(index) or isinstance(index[i], slice)]
        if np.ndim(sub) == 0:
            return ProcessMesh([int(sub)], ['d0'])
        return ProcessMesh(sub, names[:np.ndim(sub)])

    def axis_group(self, dim):
        """Communication group of this rank along mesh dim `dim` (all ranks sharing the other
        coordinates). Every rank creates every group of the axis in the same order, as
        torch.distributed requires, then keeps its own."""
        axis = self._dim(dim)
        key = (tuple(self.process_ids), tuple(self.shape), axis)
        if key not in _axis_groups:
            moved = np.moveaxis(self._mesh, axis, -1).reshape(-1, self._mesh.shape[axis])
            mine = None
            me = C.get_rank()
            for ranks in moved:
                ranks = [int(r) for r in ranks]
                g = C.new_group(ranks) if len(ranks) > 1 and C.get_world_size() > 1 else None
                if me in ranks:
                    mine = g
            _axis_groups[key] = mine
        return _axis_groups[key]

    def __enter__(self):
        _mesh_stack.append(self)
        return self

    def __exit__(self, *exc):
        _mesh_stack.pop()

    def __eq__(self, other):
        return isinstance(other, ProcessMesh) and self.shape == other.shape and \
            self.process_ids == other.process_ids

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash((tuple(self.shape), tuple(self.process_ids)))

    def __deepcopy__(self, memo):
        return ProcessMesh(self._mesh.copy(), list(self._dim_names))

    def __str__(self):
        return f"{{shape: {self.shape}, process_ids: {self.process_ids}, dim_names: {self._dim_names}}}"

    __repr__ = __str__


def get_current_process_mesh():
    return _mesh_stack[-1] if _mesh_stack else None


def _world_mesh():
    return ProcessMesh(list(range(C.get_world_size())), ['x'])


# ============================================================================================
# Dist attributes
# ============================================================================================
class DistAttr:
    """Placement of a tensor: `dims_mapping[i]` = mesh dim tensor dim i is split over (-1 = not)."""

    def __init__(self, process_mesh, dims_mapping, global_shape):
        self.process_mesh = process_mesh
        self.dims_mapping = list(dims_mapping)
        self.global_shape = list(global_shape)

    @property
    def shard_spec(self):
        n = self.process_mesh.dim_names
        return [None if d < 0 else n[d] for d in self.dims_mapping]

    def local_shape(self):
        s = list(self.global_shape)
        for i, d in enumerate(self.dims_mapping):
            if d >= 0:
                s[i] //= self.process_mesh.shape[d]
        return s

    def __repr__(self):
        return f"DistAttr(mesh={self.process_mesh}, dims_mapping={self.dims_mapping}, global_shape={self.global_shape})"


def dist_attr(x):
    return getattr(x, '_dist_attr', None)


def _spec_to_mapping(shard_spec, shape, mesh):
    if shard_spec is None:
        return [-1] * len(shape)
    assert isinstance(shard_spec, (list, tuple)), f"shard_spec {shard_spec} must be a list"
    assert len(shard_spec) == len(shape), f"shard_spec {shard_spec} needs one entry per dim of {shape}"
    mapping, used = [], set()
    for i, name in enumerate(shard_spec):
        if name is None:
            mapping.append(-1)
            continue
        assert name in mesh.dim_names, f"shard_spec entry {name!r} is not a dim of {mesh}"
        d = mesh.dim_names.index(name)
        assert d not in used, f"mesh dim {name!r} used twice in {shard_spec}"
        assert shape[i] % mesh.shape[d] == 0, \
            f"tensor dim {i} ({shape[i]}) not divisible by mesh dim {name!r} ({mesh.shape[d]})"
        used.add(d)
        mapping.append(d)
    return mapping


def _local_slice(t, attr):
    coord = attr.process_mesh.coord()
    if coord is None:
        return t[tuple(slice(0, 0) for _ in t.shape)] if t.dim() else t
    for i, d in enumerate(attr.dims_mapping):
        if d >= 0:
            n = t.shape[i] // attr.process_mesh.shape[d]
            t = t.narrow(i, coord[d] * n, n)
    return t


class _GatherAxis(torch.autograd.Function):
    """all_gather along one mesh axis, concatenated on tensor dim `dim`; backward keeps the
    local chunk (the consumer computes the same replicated loss on every rank of the axis)."""

    @staticmethod
    def forward(ctx, t, dim, group):
        ctx.dim, ctx.n, ctx.rank = dim, group.nranks, group.rank
        parts = [torch.empty_like(t) for _ in range(group.nranks)]
        torch.distributed.all_gather(parts, t.contiguous(), group=group.process_group)
        return torch.cat(parts, dim)

    @staticmethod
    def backward(ctx, g):
        n = g.shape[ctx.dim] // ctx.n
        return g.narrow(ctx.dim, ctx.rank * n, n).contiguous(), None, None


def _to_global(t, attr):
    mesh = attr.process_mesh
    if mesh.coord() is None:
        return t
    for i, d in enumerate(attr.dims_mapping):
        if d >= 0:
            g = mesh.axis_group(d)
            if g is not None:
                t = _GatherAxis.apply(t, i, g)
    return t


def _attach(x, attr):
    x._dist_attr = attr
    return x


# ============================================================================================
# Public annotation API
# ============================================================================================
def shard_tensor(x, process_mesh=None, shard_spec=None):
    """Place `x` on `process_mesh`: tensor dim i is split over mesh dim `shard_spec[i]`
    (reference interface.py:28). Returns a Tensor holding this rank's shard (a Parameter keeps
    its identity and has its data replaced by the shard, so optimizers built later see it)."""
    mesh = process_mesh or get_current_process_mesh()
    assert mesh is not None, "shard_tensor needs a process_mesh (argument or `with mesh:`)"
    assert isinstance(mesh, ProcessMesh), f"process_mesh {mesh} is not a ProcessMesh"
    from ...static import _STATIC
    from ...static.graph import Variable
    if isinstance(x, Variable) or (_STATIC[0] and isinstance(x, Parameter)):
        # static program: annotate only; the Partitioner builds this rank's program
        from .static_passes import annotate
        return annotate(x, mesh, shard_spec)
    if isinstance(x, np.ndarray):
        x = Tensor(torch.as_tensor(x))
    elif not isinstance(x, Tensor):
        x = Tensor(torch.as_tensor(x))
    t = _u(x)
    old = dist_attr(x)
    if old is not None:  # already placed: move it
        return reshard(x, mesh, shard_spec)
    attr = DistAttr(mesh, _spec_to_mapping(shard_spec, list(t.shape), mesh), list(t.shape))
    local = _local_slice(t.detach() if isinstance(x, Parameter) else t, attr).contiguous()
    if isinstance(x, Parameter):
        x._t.data = local.clone()
        return _attach(x, attr)
    out = Tensor(local)
    out.stop_gradient = x.stop_gradient
    return _attach(out, attr)


def reshard(x, process_mesh, shard_spec=None):
    """Move a dist tensor to a new placement: gather the sharded mesh axes, slice for the new
    spec (autograd-aware: gradients flow back to the source shard)."""
    attr = dist_attr(x)
    t = _u(x)
    if attr is None:
        glob = t
    else:
        assert attr.process_mesh == process_mesh or attr.process_mesh.coord() is not None, \
            "reshard across disjoint meshes is not supported"
        glob = _to_global(t, attr)
    new = DistAttr(process_mesh, _spec_to_mapping(shard_spec, list(glob.shape), process_mesh),
                   list(glob.shape))
    out = Tensor(_local_slice(glob, new).contiguous())
    out.stop_gradient = getattr(x, 'stop_gradient', True)
    return _attach(out, new)


def to_global(x):
    """Full (replicated) value of a dist tensor on every rank of its mesh."""
    attr = dist_attr(x)
    return x if attr is None else Tensor(_to_global(_u(x), attr))


def shard_op(op, process_mesh=None, in_shard_specs=None, out_shard_specs=None):
    """Wrap `op` so its Tensor inputs are resharded to `in_shard_specs` before the call and its
    outputs carry `out_shard_specs` (reference interface.py shard_op). An output produced from
    local shards is annotated as is; a replicated output is sharded to the requested spec."""
    mesh = process_mesh or get_current_process_mesh()

    def wrapped(*args, **kwargs):
        m = mesh or get_current_process_mesh()
        args = list(args)
        if in_shard_specs is not None:
            ti = [i for i, a in enumerate(args) if isinstance(a, Tensor)]
            assert len(in_shard_specs) == len(ti), "one in_shard_spec per Tensor input"
            for i, spec in zip(ti, in_shard_specs):
                if spec is not None or dist_attr(args[i]) is not None:
                    args[i] = reshard(args[i], m, spec)
        out = op(*args, **kwargs)
        if out_shard_specs is None:
            return out
        outs = out if isinstance(out, (list, tuple)) else [out]
        assert len(outs) == len(out_shard_specs), "one out_shard_spec per output"
        res = []
        for o, spec in zip(outs, out_shard_specs):
            if spec is None or not isinstance(o, Tensor):
                res.append(o)
                continue
            if dist_attr(o) is not None:
                res.append(o)
            elif any(s is not None for s in spec):
                res.append(shard_tensor(o, m, spec))
            else:
                res.append(_attach(o, DistAttr(m, [-1] * o.ndim, list(o.shape))))
        return type(out)(res) if isinstance(out, (list, tuple)) else res[0]

    return wrapped


_RC_IDS = iter(range(1, 1 << 62))


def recompute(op):
    """Activation recomputation of `op` (a callable or Layer) in the backward pass. Eagerly it
    runs under ``parallel.recompute``; while a static program records, the ops of each call are
    tagged as one recompute region (``recompute_id``), which the static Engine's
    ``auto_parallel_recompute`` pass turns into a recompute segment (reference
    auto_parallel/interface.py recompute -> op attr 'recompute_id')."""
    from ...parallel.recompute import recompute as _rc

    class _RC:
        def __init__(self, f):
            self.f = f

        def __call__(self, *args, **kwargs):
            from ...static import _STATIC
            if _STATIC[0]:
                from ...static import graph as G
                prev = G._RECOMPUTE_ID[0]
                G._RECOMPUTE_ID[0] = next(_RC_IDS)
                try:
                    return self.f(*args, **kwargs)
                finally:
                    G._RECOMPUTE_ID[0] = prev
            return _rc(self.f, *args, **kwargs)

        def __getattr__(self, name):
            return getattr(self.f, name)
    return _RC(op)


def fetch(tensor, name=None, logging=False):
    """Register `tensor` to be returned (and optionally logged) by the Engine's step outputs."""
    _fetches[name or f"fetch_{len(_fetches)}"] = (tensor, logging)
    return tensor


from .strategy import Strategy  # noqa: E402
from .engine import Engine  # noqa: E402
from .static_passes import DistributedContext, Completer, Partitioner, parallelize  # noqa: E402
