"""Static-mode semi-automatic parallelism: annotate a serial Program, complete the placement of
every variable, partition it into this rank's Program (parity: the reference's
python/paddle/distributed/auto_parallel/{dist_context.py, completion.py, partitioner.py,
reshard.py} and the per-operator SPMD rules under auto_parallel/operators/dist_*.py).

Flow (what the reference's Parallelizer does for a static program)::

    with program_guard(main):                       # serial program, global shapes
        x = static.data('x', [B, H]); ... loss = ...
        shard_tensor(x, mesh, ['dp', None])         # annotations only in static mode
        shard_tensor(fc1.weight, mesh, [None, 'mp'])
    ctx = DistributedContext(main, mesh)
    Completer(ctx).complete_forward_annotation()    # placement of every variable / op
    dist_main, vmap = Partitioner(ctx).partition()  # this rank's program, local shapes
    with program_guard(dist_main): opt.minimize(vmap[loss])   # backward + update as usual

Placement is a ``dims_mapping`` per tensor dim (-1 replicated, d = split over mesh dim d).
Completion walks the forward ops once and applies a per-op rule: elementwise ops merge their
operands' mappings (broadcast from the right; a python-scalar operand keeps the tensor's),
matmul / linear take batch dims from x and the output column from the weight and turn a
contraction dim split on both sides into a PARTIAL sum, reductions over a split dim are partial,
softmax / layer_norm / cross-entropy need their normalised axis whole, transpose permutes, an
embedding with a hidden-split table yields hidden-split rows, everything else runs replicated.

Partitioning re-records each op in a new Program through the normal static recording (so shape
inference yields the local shapes) and inserts the communication the placements imply:
  * ``ap_allreduce`` after an op with a partial output (forward all-reduce over the mesh dim,
    backward identity: row-parallel linear, a sum over a split batch);
  * ``ap_identity`` on an input that is replicated over a mesh dim the op's output is split over
    (forward identity, backward all-reduce: the column-parallel input of Megatron, and every
    replicated parameter of a data-parallel step -- this is the gradient all-reduce);
  * ``ap_gather`` / ``ap_slice`` where a consumer needs another placement than the producer
    gave (reshard: all-gather along the mesh dim, backward keeps the local slice / the reverse);
  * data variables are fed whole on every rank and sliced in the program; parameters become
    local shards of the initialised serial values; a row-parallel linear's bias is added after
    the all-reduce (once, not once per rank).
Collectives run over ProcessMesh.axis_group (RCCL on the device, gloo on the host).
"""
import numpy as np
import torch

from ...framework.core import Parameter, Tensor, _u
from ...static import graph as G
from . import ProcessMesh, _GatherAxis

__all__ = ['DistributedContext', 'Completer', 'Partitioner', 'annotate', 'parallelize']




# ----------------------------------------------------------------------------- comm ops
# Each runs through the static recorder (meta tensors during shape inference: no collective
# then) and through the Executor (real tensors, torch.distributed over the mesh-axis group).

class _AllReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, group, avg):
        ctx.scale = 1.0 / group.nranks if avg else 1.0
        t = t.clone()
        if not t.is_meta:
            torch.distributed.all_reduce(t, group=group.process_group)
            if avg:
                t.mul_(ctx.scale)
        return t

    @staticmethod
    def backward(ctx, g):
        return (g * ctx.scale if ctx.scale != 1.0 else g), None, None


class _Identity(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, group):
        ctx.group = group
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        torch.distributed.all_reduce(g, group=ctx.group.process_group)
        return g, None


class _Slice(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dim, group):
        ctx.dim, ctx.group = dim, group
        n = t.shape[dim] // group.nranks
        if not t.is_meta:
            assert n * group.nranks == t.shape[dim], \
                f"dim {dim} of size {t.shape[dim]} does not split over {group.nranks} ranks"
        return t.narrow(dim, group.rank * n, n).contiguous()

    @staticmethod
    def backward(ctx, g):
        parts = [torch.empty_like(g) for _ in range(ctx.group.nranks)]
        torch.distributed.all_gather(parts, g.contiguous(), group=ctx.group.process_group)
        return torch.cat(parts, ctx.dim), None, None


def _ap_allreduce(x, mesh, d, avg=False):
    g = mesh.axis_group(d)
    return Tensor(_AllReduce.apply(_u(x), g, avg)) if g is not None else x


def _ap_identity(x, mesh, d):
    g = mesh.axis_group(d)
    return Tensor(_Identity.apply(_u(x), g)) if g is not None else x


def _ap_gather(x, dim, mesh, d):
    g = mesh.axis_group(d)
    if g is None:
        return x
    t = _u(x)
    if t.is_meta:
        return Tensor(torch.cat([t] * g.nranks, dim))
    return Tensor(_GatherAxis.apply(t, dim, g))


def _ap_slice(x, dim, mesh, d):
    g = mesh.axis_group(d)
    return Tensor(_Slice.apply(_u(x), dim, g)) if g is not None else x


_COMM = {'ap_allreduce': _ap_allreduce, 'ap_identity': _ap_identity, 'ap_gather': _ap_gather,
         'ap_slice': _ap_slice}
for _n, _f in _COMM.items():
    G.register_static_op(_n, _f)


def _comm(name, *args):
    """Record a comm op (also when its operand is a Parameter, which static_op would run eagerly)."""
    return G.record_op(name, _COMM[name], list(args), {})


# ----------------------------------------------------------------------------- context

def _key(t):
    if isinstance(t, (G.Variable, G._VarRef)):
        return ('v', t.vid)
    return ('p', id(t))


def _ndim(t, prog):
    if isinstance(t, G._VarRef):
        t = G._ALL_VARS[t.vid]
    return len(t.shape)


def annotate(t, mesh, shard_spec):
    """Record the placement of a static Variable or a Parameter in the current program
    (``shard_tensor`` does this in static mode instead of slicing)."""
    from . import _spec_to_mapping
    prog = G.default_main_program()
    full = int(np.prod(mesh.shape))
    shape = [s if s >= 0 else full for s in t.shape]   # unknown dims: checked when fed
    mapping = _spec_to_mapping(shard_spec, shape, mesh)
    prog.__dict__.setdefault('_dist_annotations', {})[_key(t)] = (mesh, mapping, t)
    if isinstance(t, Parameter):
        # a parameter may be annotated where the model is built and used in another program
        # (auto_parallel.Engine records its own): the placement travels with the parameter
        t.__dict__['_pra_placement'] = (mesh, list(mapping))
    return t


class DistributedContext:
    """Placements of a serial program's tensors on one process mesh (reference
    python/paddle/distributed/auto_parallel/dist_context.py:51 DistributedContext). ``mapping[key]`` = dims_mapping; ``plans`` = per
    forward op the operand placements it runs with, its output placements and its partial
    (pending all-reduce) mesh dims."""

    def __init__(self, program=None, mesh=None):
        self.program = program or G.default_main_program()
        ann = dict(self.program.__dict__.get('_dist_annotations', {}))
        for p in self.program._params.values():
            pl = p.__dict__.get('_pra_placement')
            if pl is not None and _key(p) not in ann:
                ann[_key(p)] = (pl[0], pl[1], p)
        if mesh is None:
            meshes = {hash(m): m for m, _, _ in ann.values()}
            assert len(meshes) <= 1, "one process mesh per program"
            mesh = next(iter(meshes.values())) if meshes else ProcessMesh([0], ['x'])
        self.mesh = mesh
        self.mapping = {k: list(m) for k, (_, m, _) in ann.items()}
        self.annotated = set(self.mapping)
        self.plans = []

    def get(self, t):
        k = _key(t)
        if k not in self.mapping:
            self.mapping[k] = [-1] * _ndim(t, self.program)
        return self.mapping[k]

    def dims_mapping(self, t):
        return list(self.get(t))

    def shard_spec(self, t):
        names = self.mesh.dim_names
        return [None if d < 0 else names[d] for d in self.get(t)]


# ----------------------------------------------------------------------------- completion

_UNARY = {'relu', 'gelu', 'tanh', 'sigmoid', 'silu', 'exp', 'log', 'sqrt', 'square', 'abs', 'neg',
          'scale', 'dropout', 'cast', 'astype', 'clip', 'leaky_relu', 'relu6', 'swish', 'softplus',
          'erf', 'rsqrt', 'sin', 'cos', 'pow', 'hardswish', 'mish', 'elu', 'selu'}
_BINARY = {'add', 'subtract', 'multiply', 'divide', 'maximum', 'minimum'}
_LAST_AXIS = {'softmax', 'log_softmax', 'layer_norm', 'rms_norm'}
_CLASS_LOSS = {'cross_entropy', 'softmax_with_cross_entropy'}
_PAIR_LOSS = {'mse_loss', 'l1_loss', 'smooth_l1_loss'}
_REDUCE = {'sum': (1, 3), 'mean': (1, 2)}    # positions of axis / keepdim


def _arg(op, i, name, default=None):
    return op.args[i] if len(op.args) > i else op.kwargs.get(name, default)


def _tensor_args(op):
    """(position, operand) of an op's top-level tensor operands (Variables as _VarRef,
    Parameters); nested operands (lists of tensors) always run replicated."""
    out = [(i, a) for i, a in enumerate(op.args) if isinstance(a, (G._VarRef, Tensor))]
    out += [(k, a) for k, a in op.kwargs.items() if isinstance(a, (G._VarRef, Tensor))]
    return out


def _merge(ms, nd):
    """Broadcast-merge operand mappings (aligned from the right) into an output of rank nd."""
    res = [-1] * nd
    for m in ms:
        for j in range(1, len(m) + 1):
            if m[-j] >= 0 and res[-j] < 0 and m[-j] not in res:
                res[-j] = m[-j]
    return res


def _align(out, nd_in):
    """The mapping an operand of rank nd_in takes to combine (broadcast) with output `out`."""
    return [out[len(out) - nd_in + i] for i in range(nd_in)]


class Completer:
    """Forward placement completion (reference auto_parallel/completion.py:107 Completer,
    :936 complete_forward_annotation): one pass over the
    forward ops in program order, each op's SPMD rule mapping operand placements to the
    placements it runs with and produces."""

    def __init__(self, ctx):
        self.ctx = ctx

    def complete_forward_annotation(self, program=None):
        ctx = self.ctx
        prog = program or ctx.program
        vars_ = prog.global_block().vars
        seen = set()
        for op in prog.global_block().ops:
            if op.role != 'forward':
                continue
            name = op.type.rsplit(':', 1)[-1]
            targs = _tensor_args(op)
            ins = [list(ctx.get(a)) for _, a in targs]
            nd_out = [len(vars_[v].shape) for v in op.out_vids]
            req, outs, partial = self._rule(name, op, ins, nd_out)
            for (_, a), want in zip(targs, req):
                # a parameter nobody annotated takes the placement its first consumer runs
                # with (the column-parallel bias becomes a shard, not a sliced replica)
                if isinstance(a, Parameter) and _key(a) not in ctx.annotated and _key(a) not in seen:
                    ctx.mapping[_key(a)] = list(want)
                seen.add(_key(a))
            ctx.plans.append((op, req, outs, partial))
            for v, m in zip(op.out_vids, outs):
                ctx.mapping[('v', v)] = list(m)
        return ctx

    @staticmethod
    def _replicated(ins, nd_out):
        return [[-1] * len(m) for m in ins], [[-1] * n for n in nd_out], {}

    def _rule(self, name, op, ins, nd_out):
        one = len(nd_out) == 1
        if name in ('linear', 'matmul') and len(ins) >= 2 and one:
            x, w = ins[0], ins[1]
            tx = name == 'matmul' and bool(_arg(op, 2, 'transpose_x', False))
            ty = name == 'matmul' and bool(_arg(op, 3, 'transpose_y', False))
            if len(w) != 2 or len(x) < 2 or tx:
                return self._replicated(ins, nd_out)
            wk, wn = (w[1], w[0]) if ty else (w[0], w[1])
            out = list(x[:-1]) + [wn]
            if wn >= 0 and wn in out[:-1]:          # mesh dim used twice: gather the weight column
                wn = out[-1] = -1
            partial = {}
            if wk < 0 or wk in out:                  # contraction runs whole
                wk = -1
            else:                                    # contraction split on x and w: partial sum
                partial = {wk: 'sum'}
            req = [list(x[:-1]) + [wk], [wn, wk] if ty else [wk, wn]]
            for extra in ins[2:]:                    # bias follows the output column
                req.append([out[-1]] if len(extra) == 1 else [-1] * len(extra))
            return req, [out], partial
        if name in _UNARY and ins and one:
            return [ins[0]] + [[-1] * len(o) for o in ins[1:]], [list(ins[0])], {}
        if name in _BINARY and len(ins) == 2 and one:
            out = _merge(ins, nd_out[0])
            return [_align(out, len(i)) for i in ins], [out], {}
        if name in _BINARY and len(ins) == 1 and one and len(ins[0]) == nd_out[0]:
            return [list(ins[0])], [list(ins[0])], {}      # tensor (op) python scalar
        if name == 'embedding' and len(ins) >= 2 and one:
            ids, w = ins[0], ins[1]
            if len(w) == 2 and w[0] < 0 and (w[1] < 0 or w[1] not in ids):
                # hidden-split table: each rank looks up its columns for the ids it holds
                return [list(ids), list(w)], [list(ids) + [w[1]]], {}
            return self._replicated(ins, nd_out)
        if name in _REDUCE and len(ins) == 1 and one:
            x, nd = ins[0], len(ins[0])
            ia, ik = _REDUCE[name]
            axis, keep = _arg(op, ia, 'axis'), bool(_arg(op, ik, 'keepdim', False))
            axes = list(range(nd)) if axis is None else ([axis] if isinstance(axis, int) else list(axis))
            axes = [a % nd for a in axes] if nd else []
            red = 'avg' if name == 'mean' else 'sum'
            partial = {x[a]: red for a in axes if x[a] >= 0}
            out = [(-1 if i in axes else x[i]) for i in range(nd) if keep or i not in axes]
            if len(out) != nd_out[0]:
                return self._replicated(ins, nd_out)
            return [x], [out], partial
        if name in _LAST_AXIS and ins and one:
            x = list(ins[0])
            axis = _arg(op, 1, 'axis', -1) if name in ('softmax', 'log_softmax') else -1
            if not isinstance(axis, int) or axis % len(x) != len(x) - 1:
                return self._replicated(ins, nd_out)
            x[-1] = -1
            return [x] + [[-1] * len(o) for o in ins[1:]], [x], {}
        if name in _CLASS_LOSS and len(ins) >= 2 and one:
            x = list(ins[0])
            x[-1] = -1
            lbl = [x[i] if i < len(x) - 1 else -1 for i in range(len(ins[1]))]
            return self._loss(op, x, [x, lbl] + [[-1] * len(o) for o in ins[2:]], nd_out, 4,
                              x[:-1])
        if name in _PAIR_LOSS and len(ins) >= 2 and one:
            x = _merge(ins[:2], len(ins[0]))
            return self._loss(op, x, [x, _align(x, len(ins[1]))], nd_out, 2, x)
        if name == 'transpose' and len(ins) == 1 and one:
            perm = _arg(op, 1, 'perm')
            return [ins[0]], [[ins[0][p] for p in perm]], {}
        return self._replicated(ins, nd_out)

    def _loss(self, op, x, req, nd_out, ridx, none_out):
        reduction = _arg(op, ridx, 'reduction', 'mean')
        if reduction == 'none':
            return (req, [none_out], {}) if len(none_out) == nd_out[0] else \
                self._replicated(req, nd_out)
        red = 'avg' if reduction == 'mean' else 'sum'
        return req, [[-1] * nd_out[0]], {d: red for d in x if d >= 0}


# ----------------------------------------------------------------------------- partitioner

def _local_param(p, mapping, mesh):
    t = _u(p).detach()
    coord = mesh.coord()
    for i, d in enumerate(mapping):
        if d >= 0:
            n = t.shape[i] // mesh.shape[d]
            t = t.narrow(i, coord[d] * n, n)
    lp = Parameter(t.contiguous().clone(), trainable=p.trainable, name=p.name)
    lp.__dict__['_dist_mapping'] = list(mapping)
    return lp


def _needs_grad(a):
    if isinstance(a, Parameter):
        return bool(a.trainable)
    if isinstance(a, G._VarRef):
        return not G._ALL_VARS[a.vid].stop_gradient
    return False


class Partitioner:
    """This rank's program from a completed serial program (reference auto_parallel/
    partitioner.py:38 Partitioner / :69 partition for the local shapes / parameters,
    reshard.py:1006 Resharder / :2672 reshard for the inserted communication). ``partition()``
    returns ``(program, var_map)``: ``var_map[serial_var]`` is its local Variable."""

    def __init__(self, ctx, rank=None):
        self.ctx = ctx
        self.params = {}
        self.param_dims = {}   # local parameter name -> its serial parameter's dims mapping

    def local_param(self, p):
        """The local shard of serial Parameter `p` in the partitioned program."""
        return self.params[id(p)]

    def _param(self, p):
        if id(p) not in self.params:
            self.params[id(p)] = _local_param(p, self.ctx.get(p), self.ctx.mesh)
            self.param_dims[self.params[id(p)].name] = list(self.ctx.get(p))
        return self.params[id(p)]

    def _reshard(self, val, have, want):
        """`val` placed as `have` -> placed as `want`: all-gather the mesh dims it must lose,
        slice the ones it must gain."""
        mesh, have = self.ctx.mesh, list(have)
        for i, (h, w) in enumerate(zip(have, want)):
            if h >= 0 and h != w:
                val, have[i] = _comm('ap_gather', val, i, mesh, h), -1
        for i, (h, w) in enumerate(zip(have, want)):
            if w >= 0 and h != w:
                val, have[i] = _comm('ap_slice', val, i, mesh, w), w
        return val

    def _operand(self, a, want, vmap):
        if isinstance(a, G._VarRef):
            return self._reshard(vmap[a.vid], self.ctx.get(a), want)
        if isinstance(a, Parameter):
            return self._reshard(self._param(a), self.ctx.get(a), want)
        return a                                     # a constant tensor: replicated as is

    def _nested(self, obj, vmap):
        if isinstance(obj, (G._VarRef, Parameter)):
            return self._operand(obj, [-1] * _ndim(obj, None), vmap)
        if isinstance(obj, list):
            return [self._nested(o, vmap) for o in obj]
        if isinstance(obj, tuple):
            return tuple(self._nested(o, vmap) for o in obj)
        if isinstance(obj, dict):
            return {k: self._nested(v, vmap) for k, v in obj.items()}
        return obj

    def partition(self, program=None):
        ctx, mesh = self.ctx, self.ctx.mesh
        serial = program or ctx.program
        if not ctx.plans:
            Completer(ctx).complete_forward_annotation(serial)
        dist, vmap = G.Program(), {}
        sync = {}   # local parameter name -> mesh dims its gradient is all-reduced over
        with G.program_guard(dist):
            for vid, v in list(serial.global_block().vars.items()):
                if v.__dict__.get('is_data'):
                    nv = G.data(v.name, list(v.shape), v.dtype)
                    nv.stop_gradient = v.stop_gradient
                    m = ctx.get(v)
                    vmap[vid] = self._reshard(nv, [-1] * len(m), m)
            def grad_dims(op, partial, outs, pos, want):
                # replicated over a mesh dim the op's result is split / partial over: the
                # operand's gradient is a partial sum there (identity fwd, all-reduce bwd; a
                # bias added after the all-reduce only sees the split dims)
                name = op.type.rsplit(':', 1)[-1]
                split_dims = {d for m in outs for d in m if d >= 0}
                bias_pos = None
                if partial and name == 'linear':
                    bias_pos = 2 if len(op.args) > 2 else ('bias' if 'bias' in op.kwargs else None)
                dims = split_dims if pos == bias_pos else split_dims | set(partial)
                return frozenset(dims - {w for w in want if w >= 0})
            # Parameters whose every use needs the same gradient reduction (the data-parallel
            # case): no per-use identity op; their gradients are all-reduced in flat buckets,
            # asynchronously, inside the backward (meta_optimizers.insert_grad_sync at minimize)
            uses = {}
            for op, req, outs, partial in ctx.plans:
                for (pos, a), want in zip(_tensor_args(op), req):
                    if isinstance(a, Parameter) and _needs_grad(a):
                        uses.setdefault(id(a), set()).add(grad_dims(op, partial, outs, pos, want))
            deferred = {pid: next(iter(ds)) for pid, ds in uses.items() if len(ds) == 1 and next(iter(ds))}
            prev_rc = G._RECOMPUTE_ID[0]
            for op, req, outs, partial in ctx.plans:
                # the op's recompute region covers its resharding / partial-sum communication too
                G._RECOMPUTE_ID[0] = op.attrs.get('recompute_id')
                name = op.type.rsplit(':', 1)[-1]
                top = (G._VarRef, Tensor)            # top-level operands: placed by the plan below
                args = [a if isinstance(a, top) else self._nested(a, vmap) for a in op.args]
                kw = {k: a if isinstance(a, top) else self._nested(a, vmap) for k, a in op.kwargs.items()}
                bias_pos = None
                if partial and name == 'linear':     # a row-parallel bias goes after the all-reduce
                    bias_pos = 2 if len(op.args) > 2 else ('bias' if 'bias' in op.kwargs else None)
                bias = None
                for (pos, a), want in zip(_tensor_args(op), req):
                    val = self._operand(a, want, vmap)
                    if _needs_grad(a):
                        if isinstance(a, Parameter) and id(a) in deferred:
                            sync[self._param(a).name] = sorted(deferred[id(a)])
                        else:
                            for d in sorted(grad_dims(op, partial, outs, pos, want)):
                                val = _comm('ap_identity', val, mesh, d)
                    if pos == bias_pos:
                        bias, val = val, None
                    if isinstance(pos, int):
                        args[pos] = val
                    else:
                        kw[pos] = val
                res = G.record_op(op.type, op.fn, args, kw)
                flat, _ = G._flatten_out(res)
                for d, red in sorted(partial.items()):
                    flat = [_comm('ap_allreduce', f, mesh, d, red == 'avg') for f in flat]
                if bias is not None:
                    flat = [f + bias for f in flat]
                for ov, nv in zip(op.out_vids, flat):
                    vmap[ov] = nv
            G._RECOMPUTE_ID[0] = prev_rc
        dist.__dict__['_dist_context'] = ctx
        dist.__dict__['_ap_param_dims'] = dict(self.param_dims)
        dist.__dict__['_ap_mesh'] = mesh
        if sync:
            groups = {d: mesh.axis_group(d) for ds in sync.values() for d in ds}
            dist.__dict__['_ap_grad_sync'] = {n: [groups[d] for d in ds if groups[d] is not None]
                                              for n, ds in sync.items()}
        return dist, _VarMap(vmap)


class _VarMap(dict):
    """serial vid -> local Variable; also indexable by the serial Variable itself."""

    def __getitem__(self, k):
        return dict.__getitem__(self, k.vid if isinstance(k, G.Variable) else k)


def parallelize(program=None, mesh=None):
    """Complete + partition: ``(dist_program, var_map, partitioner)``."""
    ctx = DistributedContext(program, mesh)
    Completer(ctx).complete_forward_annotation()
    part = Partitioner(ctx)
    dist, vmap = part.partition()
    return dist, vmap, part
