"""Static graph: Program / Variable / OpDesc / Executor (parity: python/paddle/fluid/framework.py
(Program, Block, Variable, Operator), python/paddle/fluid/executor.py (Executor),
python/paddle/fluid/backward.py (append_backward, gradients), python/paddle/static/io.py
(save/load_inference_model), paddle/fluid/framework/new_executor/* (interpreter)).

MI355X design. Under ``paddle.enable_static()`` every ``paddle.*`` / ``F.*`` call that
touches a symbolic ``Variable`` is RECORDED as an ``OpDesc`` (qualified op name +
argument template); output shapes/dtypes are inferred by running the very same op on
``meta`` tensors (no separate InferMeta tables to drift). ``Executor.run`` replays the
program through the same kernel registry (HIP kernels / hipBLASLt / MIOpen) in the
order chosen by the native C++ scheduler (``native/src/graph_scheduler.cpp``:
dependency DAG, dead-op pruning against the fetch list, last-use GC points), with
optional HIP-graph capture of the whole replay for static shapes.

Backward is part of the IR (parity: python/paddle/fluid/backward.py:1826 append_backward):
``append_backward`` walks the forward ops in reverse and emits one ``<type>_grad`` OpDesc
per differentiable op (reading the forward op's saved context var and its output grads,
writing its input / parameter grads), ``sum`` ops where a var or parameter feeds several
ops, and a ``fill_grad_seed`` op for the loss. At replay each forward op that has a grad op
runs on leaf copies of its inputs and keeps its OWN small autograd graph in the context
var; its grad op differentiates exactly that graph (torch.autograd.grad), so dropout masks
and AMP casts match the forward. ``optimize`` consumes the ``param@GRAD`` vars. Forward +
backward of a training program can be captured as ONE HIP graph
(``BuildStrategy.use_hip_graph``); the optimizer step runs after the replay.

Serialized programs (``.pdmodel``, a framework.proto ProgramDesc written by
static/program_desc.py) name ops only by their registered op type; loading resolves names through the static op table and refuses anything else.
"""
import collections
import inspect
import contextlib
import itertools
import weakref
import json
import os
import time

import numpy as np
import torch

from ..framework.core import Tensor, Parameter, _u, convert_dtype, dtype_to_str, _default_device
from . import _STATIC

_PROBES = (3, 5)  # sizes substituted for unknown (-1) dims during meta shape inference
_var_ids = itertools.count()
_ALL_VARS = weakref.WeakValueDictionary()  # vid -> Variable, across programs / sub-blocks


# =============================================================================
# Variable / OpDesc / Program
# =============================================================================
class Variable(Tensor):
    """Symbolic tensor of a Program (static mode)."""

    def __init__(self, block, shape, dtype, name=None, persistable=False, stop_gradient=True,
                 is_data=False):
        shp = [(-1 if s is None else int(s)) for s in shape]
        meta_shape = [(_PROBES[0] if s < 0 else s) for s in shp]
        t = torch.empty(meta_shape, dtype=convert_dtype(dtype) or torch.float32, device='meta')
        object.__setattr__(self, '_t', t)
        self._name = name
        self.persistable = persistable
        self.__dict__['_vshape'] = shp
        self.__dict__['vid'] = next(_var_ids)
        self.__dict__['block'] = block
        self.__dict__['is_data'] = is_data
        self.__dict__['_sg'] = stop_gradient
        self.__dict__['op'] = None
        _ALL_VARS[self.vid] = self

    @property
    def shape(self):
        return list(self._vshape)

    @property
    def stop_gradient(self):
        return self.__dict__.get('_sg', True)

    @stop_gradient.setter
    def stop_gradient(self, v):
        self.__dict__['_sg'] = bool(v)

    @property
    def name(self):
        if self._name is None:
            self._name = f'tmp_{self.vid}'
        return self._name

    @name.setter
    def name(self, v):
        self._name = v

    @property
    def program(self):
        return self.block.program

    def __repr__(self):
        return f'var {self.name} : shape={self.shape} dtype={dtype_to_str(self.dtype)}'

    def numpy(self):
        raise RuntimeError("a static Variable has no value; fetch it with Executor.run")

    def __bool__(self):
        raise RuntimeError("static Variables have no truth value (use paddle.static.nn.cond)")

    def __hash__(self):
        return id(self)


class GradVar(Variable):
    """``param@GRAD``: resolved from the parameter's accumulated gradient after backward."""

    def __init__(self, block, param):
        super().__init__(block, list(_u(param).shape), _u(param).dtype, name=param.name + '@GRAD')
        self.__dict__['param'] = param


class _VarRef:
    __slots__ = ('vid',)

    def __init__(self, vid):
        self.vid = vid


class OpDesc:
    """One op of a Block (parity: framework.proto OpDesc: type, inputs, outputs, attrs).

    ``role`` is 'forward', 'backward' (grad / sum / seed ops from append_backward) or
    'optimize'; a forward op that has a grad op also writes a context var ``ctx_vid``."""

    def __init__(self, type, fn, args, kwargs, in_vids, out_vids, out_template, role='forward'):
        self.type, self.fn = type, fn
        self.args, self.kwargs = args, kwargs
        self.in_vids, self.out_vids = in_vids, out_vids
        self.out_template = out_template
        self.attrs = {}
        self.role = role
        self.ctx_vid = None

    def all_outputs(self):
        return self.out_vids + ([self.ctx_vid] if self.ctx_vid is not None else [])

    def __repr__(self):
        return f'{{Out={self.out_vids}}} = {self.type}(inputs={self.in_vids})'


class Block:
    def __init__(self, program, idx=0):
        self.program, self.idx = program, idx
        self.ops = []
        self.vars = {}

    def var(self, name):
        for v in self.vars.values():
            if v.name == name:
                return v
        raise ValueError(f'var {name} not found')

    def has_var(self, name):
        return any(v.name == name for v in self.vars.values())

    def all_parameters(self):
        return self.program.all_parameters()

    def create_var(self, name=None, shape=(), dtype='float32', persistable=False, **kw):
        v = Variable(self, shape, dtype, name, persistable)
        self.vars[v.vid] = v
        return v


class Program:
    _counter = itertools.count()

    def __init__(self):
        self.blocks = [Block(self, 0)]
        self.random_seed = 0
        self._version = 0
        self._params = {}  # name -> Parameter (persistables referenced by ops)
        self._plans = {}
        self._is_startup = False
        self._id = next(Program._counter)
        self._hip_graph = None

    def global_block(self):
        return self.blocks[0]

    def current_block(self):
        return self.blocks[0]

    def block(self, i):
        return self.blocks[i]

    @property
    def num_blocks(self):
        return len(self.blocks)

    def list_vars(self):
        return list(self.global_block().vars.values()) + list(self._params.values())

    def all_parameters(self):
        return list(self._params.values())

    def _register_param(self, p):
        self._params.setdefault(p.name, p)

    def clone(self, for_test=False):
        p = Program()
        ops = []
        for op in self.global_block().ops:
            if for_test and op.role != 'forward':
                continue
            if for_test:
                kw = dict(op.kwargs, training=False) if isinstance(op.kwargs, dict) and \
                    op.kwargs.get('training') is True else op.kwargs
                nop = OpDesc(op.type, op.fn, op.args, kw, op.in_vids, op.out_vids, op.out_template)
                nop.attrs = dict(op.attrs)
                op = nop
            ops.append(op)
        p.blocks[0].ops = ops
        p.blocks[0].vars = dict(self.global_block().vars)
        p._params = dict(self._params)
        p._for_test = for_test
        return p

    def state_dict(self, mode='all', scope=None):
        return {n: p for n, p in self._params.items()}

    def set_state_dict(self, state_dict, scope=None):
        for n, v in state_dict.items():
            if n in self._params:
                self._params[n].set_value(v)

    def _bump(self):
        self._version += 1
        self._plans.clear()
        self._hip_graph = None

    def __str__(self):
        lines = [f'Program {self._id}:']
        for v in self.global_block().vars.values():
            if v.is_data:
                lines.append(f'  feed  {v!r}')
        for op in self.global_block().ops:
            lines.append(f'  {op!r}')
        return '\n'.join(lines)

    to_string = lambda self, throw_on_error=False, with_details=False: str(self)  # noqa: E731


_main_program = [Program()]
_startup_program = [Program()]
_startup_program[0]._is_startup = True


def default_main_program():
    return _main_program[0]


def default_startup_program():
    return _startup_program[0]


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    prev_m, prev_s = _main_program[0], _startup_program[0]
    _main_program[0] = main_program
    if startup_program is not None:
        startup_program._is_startup = True
        _startup_program[0] = startup_program
    try:
        yield
    finally:
        _main_program[0], _startup_program[0] = prev_m, prev_s


@contextlib.contextmanager
def name_scope(prefix=None):
    yield


_DEVICE = [None]


@contextlib.contextmanager
def device_guard(device=None):
    """Ops recorded inside carry ``attrs['device']`` (parity: fluid/framework.py device_guard,
    the op_device attribute PipelineOptimizer splits a program by). A program spread over
    several GPUs trains through the static pipeline (PipelineOptimizer / fleet
    strategy.pipeline: one stage per rank, static/pipeline.py); a plain ``minimize`` raises."""
    prev = _DEVICE[0]
    _DEVICE[0] = device
    try:
        yield
    finally:
        _DEVICE[0] = prev


def _device_index(dev):
    if dev is None:
        return None
    s = str(dev)
    if ':' in s:
        kind, idx = s.split(':', 1)
        return (kind, idx)
    return (s, '0') if s in ('gpu', 'cuda') else (s, None)


def check_single_device(prog, what='minimize'):
    """Raise for a program whose ops were recorded under device_guard on more than one device."""
    devs = {op.attrs.get('device') for op in prog.global_block().ops if op.attrs.get('device')}
    keys = {_device_index(d) for d in devs}
    gpus = {k for k in keys if k and k[0] in ('gpu', 'cuda')}
    if len(gpus) > 1:
        raise NotImplementedError(
            f"{what}: the program places ops on {len(gpus)} devices with static.device_guard "
            f"({sorted(devs)}); train it as a pipeline (paddle.static.PipelineOptimizer or fleet "
            "strategy.pipeline, one rank per stage)")


def data(name, shape, dtype=None, lod_level=0):
    blk = default_main_program().global_block()
    v = Variable(blk, shape, dtype or 'float32', name=name, is_data=True)
    blk.vars[v.vid] = v
    default_main_program()._bump()
    return v


# =============================================================================
# op recording
# =============================================================================
def _has_var(obj):
    if isinstance(obj, Variable):
        return True
    if isinstance(obj, (list, tuple)):
        return any(_has_var(o) for o in obj)
    if isinstance(obj, dict):
        return any(_has_var(o) for o in obj.values())
    return False


def _template(obj, in_vids, params):
    if isinstance(obj, Variable):
        in_vids.append(obj.vid)
        return _VarRef(obj.vid)
    if isinstance(obj, Parameter) or (isinstance(obj, Tensor) and obj.persistable):
        params.append(obj)
        return obj
    if isinstance(obj, list):
        return [_template(o, in_vids, params) for o in obj]
    if isinstance(obj, tuple):
        return tuple(_template(o, in_vids, params) for o in obj)
    if isinstance(obj, dict):
        return {k: _template(v, in_vids, params) for k, v in obj.items()}
    return obj


def _materialize(obj, env):
    if isinstance(obj, _VarRef):
        return env[obj.vid]
    if isinstance(obj, list):
        return [_materialize(o, env) for o in obj]
    if isinstance(obj, tuple):
        return tuple(_materialize(o, env) for o in obj)
    if isinstance(obj, dict):
        return {k: _materialize(v, env) for k, v in obj.items()}
    return obj


def _scope_vars(block, extra=()):
    """The block's variables plus outer-block variables an op inside a sub-block reads."""
    vs = dict(block.vars)
    for vid in extra:
        if vid not in vs and vid in _ALL_VARS:
            vs[vid] = _ALL_VARS[vid]
    return vs


def _meta_env(block, probe, extra=()):
    env = {}
    for vid, v in _scope_vars(block, extra).items():
        shp = [probe if s < 0 else s for s in v._vshape]
        env[vid] = Tensor(torch.empty(shp, dtype=v.dtype, device='meta'))
    return env


def _flatten_out(out):
    if isinstance(out, Tensor):
        return [out], 'T'
    if isinstance(out, (list, tuple)):
        flat, tmpl = [], []
        for o in out:
            f, t = _flatten_out(o)
            flat += f
            tmpl.append(t)
        return flat, (type(out).__name__, tmpl)
    return [], ('C', out)


def _rebuild(tmpl, it):
    if tmpl == 'T':
        return next(it)
    kind, sub = tmpl
    if kind == 'C':
        return sub
    seq = [_rebuild(t, it) for t in sub]
    return tuple(seq) if kind == 'tuple' else seq


def _param_to_meta(obj):
    if isinstance(obj, Tensor) and not isinstance(obj, Variable):
        t = obj._t
        return Tensor(torch.empty(t.shape, dtype=t.dtype, device='meta'))
    if isinstance(obj, list):
        return [_param_to_meta(o) for o in obj]
    if isinstance(obj, tuple):
        return tuple(_param_to_meta(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _param_to_meta(v) for k, v in obj.items()}
    return obj


def record_op(op_type, fn, args, kwargs, out_specs=None):
    """Append an op to the current program. ``out_specs`` = (template, [(shape, dtype)])
    skips shape inference (control-flow ops whose output shapes are their loop vars')."""
    prog = default_main_program()
    blk = prog.global_block()
    in_vids, params = [], []
    targs = _template(list(args), in_vids, params)
    tkw = _template(dict(kwargs), in_vids, params)
    for p in params:
        if isinstance(p, Parameter):
            prog._register_param(p)
    if out_specs is not None:
        tmpl, specs = out_specs
        out_vars = []
        for shp, dt in specs:
            v = Variable(blk, list(shp), dt, stop_gradient=False)
            blk.vars[v.vid] = v
            out_vars.append(v)
        op = OpDesc(op_type, fn, targs, tkw, in_vids, [v.vid for v in out_vars], tmpl)
        op.attrs['params'] = [p for p in params if isinstance(p, Parameter)]
        _record_amp(op)
        for v in out_vars:
            v.__dict__['op'] = op
        blk.ops.append(op)
        prog._bump()
        return _rebuild(tmpl, iter(out_vars))
    # shape inference: run the op on meta tensors with two probe sizes for unknown dims
    outs = []
    for probe in _PROBES:
        prev = _STATIC[0]
        _STATIC[0] = False
        try:
            with torch.no_grad():
                try:
                    env = _meta_env(blk, probe, in_vids)
                    r = fn(*_param_to_meta(_materialize(targs, env)),
                           **_param_to_meta(_materialize(tkw, env)))
                except Exception:
                    # data-dependent op (needs values): infer on zero tensors instead
                    env = _real_probe_env(blk, probe, in_vids)
                    r = fn(*_materialize(targs, env), **_materialize(tkw, env))
        finally:
            _STATIC[0] = prev
        outs.append(r)
    flat0, tmpl = _flatten_out(outs[0])
    flat1, _ = _flatten_out(outs[1])
    out_vars = []
    for t0, t1 in zip(flat0, flat1):
        s0, s1 = list(t0._t.shape), list(t1._t.shape)
        shp = [a if a == b else -1 for a, b in zip(s0, s1)] if len(s0) == len(s1) else s0
        v = Variable(blk, shp, t0._t.dtype, stop_gradient=False)
        blk.vars[v.vid] = v
        out_vars.append(v)
    op = OpDesc(op_type, fn, targs, tkw, in_vids, [v.vid for v in out_vars], tmpl)
    op.attrs['params'] = [p for p in params if isinstance(p, Parameter)]
    _record_amp(op)
    for v in out_vars:
        v.__dict__['op'] = op
    blk.ops.append(op)
    prog._bump()
    return _rebuild(tmpl, iter(out_vars))


_RECOMPUTE_ID = [None]   # set while an auto_parallel.recompute(...)-wrapped callable records


def _record_amp(op):
    """Ops recorded inside ``paddle.amp.auto_cast`` replay under the same AMP policy (and
    carry the enclosing device_guard's device and auto_parallel.recompute region)."""
    if _DEVICE[0] is not None:
        op.attrs['device'] = _DEVICE[0]
    if _RECOMPUTE_ID[0] is not None:
        op.attrs['recompute_id'] = _RECOMPUTE_ID[0]
    from ..amp import amp_state
    st = amp_state()
    if st['enabled']:
        op.attrs['amp'] = {'dtype': st['dtype'], 'level': st['level'], 'white': set(st['white']),
                           'black': set(st['black'])}


_OP_TABLE = {}  # op type -> eager function (the only things a .pdmodel may name)


def register_static_op(name, fn):
    _OP_TABLE[name] = fn
    return fn


def static_op(name, fn):
    """Wrap an eager API function so that it records when given static Variables."""
    register_static_op(name, fn)

    def wrapper(*args, **kwargs):
        if _STATIC[0] and (_has_var(args) or _has_var(kwargs)):
            return record_op(name, fn, args, kwargs)
        return fn(*args, **kwargs)
    wrapper.__name__ = getattr(fn, '__name__', name)
    wrapper.__doc__ = getattr(fn, '__doc__', None)
    wrapper.__wrapped__ = fn
    wrapper._pra_op_name = name
    return wrapper


def _op_getitem(x, idx):
    return x[idx]


def _op_binary(name):
    from .. import tensor as T

    def f(a, b):
        return getattr(T.math, name)(a, b)
    return f


# =============================================================================
# backward: grad OpDescs (parity: python/paddle/fluid/backward.py append_backward :1826,
# gradients; paddle/fluid/framework grad op makers)
# =============================================================================
class _Ctx:
    """A forward op's saved autograd context (its leaf inputs, parameters and outputs)."""
    __slots__ = ('leaves', 'params', 'outs')

    def __init__(self, leaves, params, outs):
        self.leaves, self.params, self.outs = leaves, params, outs


def _vjp(ctx, *out_grads):
    """Generic grad kernel: differentiate the forward op's own graph."""
    targets = list(ctx.leaves) + list(ctx.params)
    pairs = [(o, g) for o, g in zip(ctx.outs, out_grads)
             if g is not None and isinstance(o, torch.Tensor) and o.requires_grad]
    if pairs:
        gs = torch.autograd.grad([o for o, _ in pairs], targets,
                                 [(_u(g) if isinstance(g, Tensor) else g).to(o.dtype) for o, g in pairs],
                                 allow_unused=True)
    else:
        gs = [None] * len(targets)
    ctx.outs = ()  # the graph is consumed: free it
    return [Tensor(g if g is not None else torch.zeros_like(t)) for g, t in zip(gs, targets)]


# Direct grad kernels (parity: python/paddle/fluid/backward.py:1276 `_append_backward_ops_`,
# which emits each forward op's REGISTERED grad op running its phi grad kernel). An op type in
# _FN_OPS is backed by a torch.autograd.Function whose forward / backward ARE the op's forward
# and grad kernels: in a program with a backward the executor runs Function.forward on a plain
# context object (no autograd graph kept alive) and the `<type>_grad` op calls
# Function.backward on that context directly (no torch.autograd re-entry). A per-type
# predicate picks this path at run time; when it declines (e.g. an AMP cast the fused kernel
# does not take) the op runs the generic autograd path and its grad op falls back to _vjp.
_FN_OPS = {}   # op type -> (autograd.Function class, predicate(torch args) -> bool)
# PRA_STATIC_DIRECT_GRAD=0: every direct-grad op takes the generic autograd path (A/B timing)
_DIRECT_GRAD = __import__('os').environ.get('PRA_STATIC_DIRECT_GRAD', '1') != '0'


# direct-grad op types whose backward folds an existing partial gradient of their first input
# into the input gradient (_fn_grad ``acc``)
# (PRA_STATIC_GRAD_FOLD=0: separate `sum` ops, A/B timing)
_ACC_DX_OPS = {'fused_linear', 'fused_mlp_gelu'} \
    if __import__('os').environ.get('PRA_STATIC_GRAD_FOLD', '1') != '0' else set()


def register_fn_op(op_type, fn_cls, pred=None):
    _FN_OPS[op_type] = (fn_cls, pred)


class _FnCtx:
    """Stand-in for torch's FunctionCtx: what a Function's forward saves, its backward reads."""

    def __init__(self, fn_cls, needs, slots, order):
        self.fn_cls, self.needs_input_grad = fn_cls, needs
        self.slots, self.order = slots, order   # positional-arg -> grad-output mapping
        self.saved_tensors = ()
        self.materialize = True
        self.out_meta = []

    def save_for_backward(self, *ts):
        self.saved_tensors = ts

    def set_materialize_grads(self, v):
        self.materialize = bool(v)

    def mark_non_differentiable(self, *a):
        pass

    def mark_dirty(self, *a):
        pass


def _fn_grad(ctx, *out_grads, acc=None):
    """`<type>_grad` of a direct-grad op: Function.backward on the saved context; generic
    autograd replay when the forward took the fallback path. ``acc`` (see _ACC_DX_OPS): the
    other partial gradient of the op's first input, folded into its input gradient -- by the
    Function itself when it can (a beta=1 GEMM into ``acc``), else by one add here."""
    if isinstance(ctx, _Ctx):
        res = _vjp(ctx, *out_grads)
        if acc is not None:
            res[0] = Tensor(_u(res[0]) + _u(acc).to(_u(res[0]).dtype))
        return res
    ctx.dx_acc = _u(acc) if acc is not None else None
    ctx.dx_acc_used = False
    gs = []
    # a Function whose backward takes None for an unused output (``none_grads_ok``) is not
    # handed a zero tensor: e.g. the residual output of add+dropout+LayerNorm in a post-LN
    # encoder, which would otherwise cost a [tokens, hidden] fill per layer
    keep_none = getattr(ctx.fn_cls, 'none_grads_ok', False)
    for g, (shp, dt, dev) in zip(out_grads, ctx.out_meta):
        if g is None:
            gs.append(torch.zeros(shp, dtype=dt, device=dev) if ctx.materialize and not keep_none else None)
        else:
            t = _u(g) if isinstance(g, Tensor) else g
            gs.append(t.to(dt) if t.dtype != dt else t)
    with torch.no_grad():
        res = ctx.fn_cls.backward(ctx, *gs)
    if not isinstance(res, tuple):
        res = (res,)
    out = []
    for key in ctx.order:
        i = ctx.slots.index(key)
        g = res[i] if i < len(res) else None
        out.append(Tensor(g) if g is not None else None)
    if acc is not None and not ctx.dx_acc_used:
        a = _u(acc)
        out[0] = Tensor(a) if out[0] is None else Tensor(_u(out[0]) + a.to(_u(out[0]).dtype))
    ctx.saved_tensors = ()
    ctx.dx_acc = None
    return out


def _sum_grads(*gs):
    t = _u(gs[0])
    for g in gs[1:]:
        t = t + _u(g).to(t.dtype)
    return Tensor(t)


def _seed(target, scale=1.0):
    return Tensor(torch.full_like(_u(target), float(scale)))


for _n, _f in (('grad', _vjp), ('sum', _sum_grads), ('fill_grad_seed', _seed)):
    register_static_op(_n, _f)


def _new_var(blk, like_shape, dtype, name=None):
    v = Variable(blk, like_shape, dtype, name=name, stop_gradient=False)
    blk.vars[v.vid] = v
    return v


# -----------------------------------------------------------------------------
# forward recomputation (parity: python/paddle/fluid/backward.py:907
# `_append_backward_ops_with_checkpoints_`, fluid/optimizer.py:6447 RecomputeOptimizer)
# -----------------------------------------------------------------------------
# Segments are op ranges between checkpoints (the reference's rule: with one checkpoint the ops up
# to and including its producer; with several, the ops from the first consumer of checkpoint i to
# the producer of checkpoint i+1, plus the head before the first segment). A segment's forward ops
# run WITHOUT keeping their autograd contexts, so their intermediate outputs are freed at their
# last forward use; when the backward reaches the segment, clones of its forward ops (role
# 'recompute', fresh output vars) re-run from the held inputs and the segment's grad ops read the
# clones' contexts. The host/device RNG state is saved at the segment's start and swapped in
# around the clones, so dropout masks (seeded from the host generator) repeat bit for bit.
_FWD_ROLES = ('forward', 'recompute')


def _rng_save():
    cpu = torch.get_rng_state()
    dev = torch.cuda.get_rng_state() if torch.cuda.is_available() and torch.cuda.is_initialized() \
        else torch.empty(0, dtype=torch.uint8)
    return Tensor(cpu), Tensor(dev)


def _rng_swap(cpu, dev):
    cur = _rng_save()
    torch.set_rng_state(_u(cpu))
    d = _u(dev)
    if d.numel():
        torch.cuda.set_rng_state(d)
    return cur


def _rng_restore(cpu, dev):
    _rng_swap(cpu, dev)


for _n, _f in (('recompute_rng_save', _rng_save), ('recompute_rng_swap', _rng_swap),
               ('recompute_rng_restore', _rng_restore)):
    register_static_op(_n, _f)


def _checkpoint_vids(checkpoints):
    out = []
    for c in checkpoints or ():
        if isinstance(c, Variable):
            out.append(c.vid)
        else:
            raise TypeError(f"checkpoints must be static Variables, got {type(c).__name__}")
    return out


def _recompute_segments(fwd, ck_vids):
    """[(lo, hi)] op-index ranges of ``fwd`` to recompute (see the block comment above)."""
    producer, first_use = {}, {}
    for i, op in enumerate(fwd):
        for v in op.in_vids:
            first_use.setdefault(v, i)
        for v in op.out_vids:
            producer[v] = i
    ck = sorted({v for v in ck_vids if v in producer}, key=lambda v: producer[v])
    if not ck:
        return []
    if len(ck) == 1:
        end = producer[ck[0]]
        return [(0, end + 1)] if end > 0 else []
    segs, prev_end = [], 0
    for a, b in zip(ck, ck[1:]):
        lo = max(first_use.get(a, producer[a] + 1), prev_end)
        hi = producer[b] + 1
        if lo < hi:
            segs.append((lo, hi))
            prev_end = hi
    if segs and segs[0][0] > 0:
        segs.insert(0, (0, segs[0][0]))
    return segs


def annotated_segments(fwd, skip=()):
    """[(lo, hi)] recompute segments from ``auto_parallel.recompute`` regions: each maximal run of
    forward ops carrying one ``recompute_id`` (single-op runs are not worth recomputing); the
    ``skip`` indices (``no_recompute_segments``) are dropped (reference auto_parallel_recompute.py
    :94 get_recompute_segments)."""
    segs, i = [], 0
    while i < len(fwd):
        rid = fwd[i].attrs.get('recompute_id')
        j = i + 1
        if rid is not None:
            while j < len(fwd) and fwd[j].attrs.get('recompute_id') == rid:
                j += 1
            if j - i > 1:
                segs.append((i, j))
        i = j
    for k in sorted(set(skip), reverse=True):
        if not 0 <= k < len(segs):
            raise ValueError(f"no_recompute_segments index {k} out of range: the program has "
                             f"{len(segs)} recompute segments")
        segs.pop(k)
    return segs


def _remap_refs(obj, remap):
    if isinstance(obj, _VarRef):
        return _VarRef(remap.get(obj.vid, obj.vid))
    if isinstance(obj, list):
        return [_remap_refs(o, remap) for o in obj]
    if isinstance(obj, tuple):
        return tuple(_remap_refs(o, remap) for o in obj)
    if isinstance(obj, dict):
        return {k: _remap_refs(v, remap) for k, v in obj.items()}
    return obj


def _emit_recompute(blk, seg_ops, ctrl_vids):
    """Append the RNG swap, the clones of ``seg_ops`` and the RNG restore; returns
    (clones by id(original op), vid remap, the forward-side RNG save op)."""
    cv = _new_var(blk, [-1], torch.uint8, 'recompute@RNG_CPU')
    dv = _new_var(blk, [-1], torch.uint8, 'recompute@RNG_DEV')
    save = OpDesc('recompute_rng_save', _rng_save, [], {}, [], [cv.vid, dv.vid],
                  ('tuple', ['T', 'T']), role='forward')
    sc = _new_var(blk, [-1], torch.uint8)
    sd = _new_var(blk, [-1], torch.uint8)
    blk.ops.append(OpDesc('recompute_rng_swap', _rng_swap, [_VarRef(cv.vid), _VarRef(dv.vid)], {},
                          [cv.vid, dv.vid] + list(ctrl_vids), [sc.vid, sd.vid],
                          ('tuple', ['T', 'T']), role='backward'))
    remap, clones, last_outs = {}, {}, [sc.vid]
    for op in seg_ops:
        nop = OpDesc(op.type, op.fn, _remap_refs(op.args, remap), _remap_refs(op.kwargs, remap),
                     [remap.get(v, v) for v in op.in_vids] + [sc.vid], [], op.out_template,
                     role='recompute')
        nop.attrs = {k: v for k, v in op.attrs.items() if k not in ('diff_in', 'diff_params')}
        nop.attrs['recompute_of'] = op
        for o in op.out_vids:
            ov = blk.vars[o]
            nv = _new_var(blk, list(ov._vshape), ov.dtype, ov.name + '@RECOMPUTE')
            remap[o] = nv.vid
            nop.out_vids.append(nv.vid)
        if nop.out_vids:
            last_outs = nop.out_vids
        clones[id(op)] = nop
        blk.ops.append(nop)
    # (no outputs: the scheduler keeps an output-less op, in program order, instead of pruning it)
    blk.ops.append(OpDesc('recompute_rng_restore', _rng_restore, [_VarRef(sc.vid), _VarRef(sd.vid)], {},
                          [sc.vid, sd.vid] + list(last_outs), [], 'C', role='backward'))
    return clones, remap, save


def _build_backward(prog, targets, inputs=(), target_grads=None, no_grad_set=None,
                    params=None, loss_scale=1.0, checkpoints=None, segments_fn=None):
    """Emit grad ops for ``targets`` w.r.t. ``inputs`` (Variables) and the trainable
    parameters. Returns ({input vid: grad var}, {param name: grad var})."""
    blk = prog.global_block()
    no_grad = {getattr(x, 'name', x) for x in (no_grad_set or ())}
    fwd = [op for op in blk.ops if op.role == 'forward']
    if segments_fn is not None:
        segs = segments_fn(fwd)
    else:
        segs = _recompute_segments(fwd, _checkpoint_vids(checkpoints)) if checkpoints else []
    seg_of = {}
    for si, (lo, hi) in enumerate(segs):
        for op in fwd[lo:hi]:
            seg_of[id(op)] = si
    clones, seg_remap, rng_saves = {}, {}, []
    req = {v.vid for v in blk.vars.values() if v.is_data and not v.stop_gradient}
    req |= {x.vid for x in inputs}
    allowed = None if params is None else {id(p) for p in params}

    def diff_params(op):
        return [p for p in op.attrs.get('params', [])
                if not p.stop_gradient and p.name not in no_grad and
                (allowed is None or id(p) in allowed)]
    for op in fwd:
        if any(i in req for i in op.in_vids) or diff_params(op):
            for o in op.out_vids:
                v = blk.vars.get(o)
                if v is not None and (v.dtype.is_floating_point or v.dtype.is_complex):
                    req.add(o)
    needed = {t.vid for t in targets}
    path = []
    for op in reversed(fwd):
        if any(o in needed for o in op.out_vids) and \
                (any(i in req for i in op.in_vids) or diff_params(op)):
            path.append(op)
            needed.update(i for i in op.in_vids if i in req)
    partial = {}
    final = {}

    def add_partial(key, gv):
        partial.setdefault(key, []).append(gv)

    def final_grad(key, name=None):
        if key in final:
            return final[key]
        gs = partial.get(key, [])
        if not gs:
            final[key] = None
        elif len(gs) == 1:
            final[key] = gs[0]
        else:
            ref = blk.vars[gs[0]]
            out = _new_var(blk, ref.shape, ref.dtype, name)
            blk.ops.append(OpDesc('sum', _sum_grads, [_VarRef(g) for g in gs], {}, list(gs),
                                  [out.vid], 'T', role='backward'))
            final[key] = out.vid
        return final[key]

    for i, t in enumerate(targets):
        if target_grads is not None and i < len(target_grads) and target_grads[i] is not None:
            add_partial(t.vid, target_grads[i].vid)
            continue
        g = _new_var(blk, t.shape, t.dtype, t.name + '@GRAD')
        blk.ops.append(OpDesc('fill_grad_seed', _seed, [_VarRef(t.vid), loss_scale], {},
                              [t.vid], [g.vid], 'T', role='backward'))
        add_partial(t.vid, g.vid)
    for op in path:
        ogs = [final_grad(o) for o in op.out_vids]
        acc_in = None
        if all(g is None for g in ogs):
            continue
        diff_in = []
        for i in op.in_vids:
            if i in req and i not in diff_in:
                diff_in.append(i)
        dps = diff_params(op)
        if not diff_in and not dps:
            continue
        si = seg_of.get(id(op))
        if si is not None and si not in seg_remap:
            lo, hi = segs[si]
            cl, seg_remap[si], save = _emit_recompute(blk, fwd[lo:hi], [g for g in ogs if g is not None])
            clones.update(cl)
            rng_saves.append((fwd[lo], save))
        xop = clones.get(id(op), op)    # the op whose context the grad op reads
        remap = seg_remap.get(si, {}) if si is not None else {}
        if xop.ctx_vid is None:
            cv = Variable(blk, [], 'float32', name=f'{op.type}@CTX')
            blk.vars[cv.vid] = cv
            xop.ctx_vid = cv.vid
        xop.attrs['diff_in'] = [remap.get(i, i) for i in diff_in]
        xop.attrs['diff_params'] = dps
        fop, op = op, xop
        outs = []
        for i in diff_in:
            v = blk.vars[i]
            outs.append(_new_var(blk, v.shape, v.dtype).vid)
        for p in dps:
            outs.append(_new_var(blk, list(_u(p).shape), _u(p).dtype).vid)
        args = [_VarRef(op.ctx_vid)] + [None if g is None else _VarRef(g) for g in ogs]
        # gradient-sum fusion: when the op's first input already has exactly one partial
        # gradient from a later consumer (a residual stream feeding both a Linear / MLP and an
        # add+LayerNorm), the grad op folds it into its input gradient (beta=1 GEMM) and the
        # separate `sum` op disappears
        if op.type in _ACC_DX_OPS and op.type in _FN_OPS and diff_in and fop.args and \
                isinstance(fop.args[0], _VarRef) and fop.args[0].vid == diff_in[0] and \
                diff_in[0] not in final and len(partial.get(diff_in[0], [])) == 1:
            acc_in = partial[diff_in[0]][0]
        gop = OpDesc(op.type + '_grad', _fn_grad if op.type in _FN_OPS else _vjp, args,
                     {'acc': _VarRef(acc_in)} if acc_in is not None else {},
                     [op.ctx_vid] + [g for g in ogs if g is not None] +
                     ([acc_in] if acc_in is not None else []), outs,
                     ('list', ['T'] * len(outs)), role='backward')
        gop.attrs['fwd'] = op
        if 'amp' in op.attrs:
            gop.attrs['amp'] = op.attrs['amp']
        blk.ops.append(gop)
        if acc_in is not None:
            partial[diff_in[0]] = []   # outs[0] now carries the folded partial as well
        for i, gv in zip(diff_in, outs[:len(diff_in)]):
            add_partial(i, gv)
        for p, gv in zip(dps, outs[len(diff_in):]):
            add_partial(('param', p.name), gv)
            prog._register_param(p)
    # each recomputed segment's RNG snapshot is taken in the forward, right before its first op
    for first, save in rng_saves:
        blk.ops.insert(blk.ops.index(first), save)
    in_grads = {x.vid: final_grad(x.vid, x.name + '@GRAD') for x in inputs}
    p_grads = {}
    for key in list(partial):
        if isinstance(key, tuple) and key[0] == 'param':
            p_grads[key[1]] = final_grad(key, key[1] + '@GRAD')
    prog._bump()
    return in_grads, p_grads


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None,
                    checkpoints=None, loss_scale=1.0, segments_fn=None):
    """Append grad ops for ``loss``; returns [(param, param@GRAD var)]. ``segments_fn(forward
    ops) -> [(lo, hi)]`` picks the recompute segments directly (annotated regions)."""
    prog = loss.block.program
    blk = prog.global_block()
    params = None
    if parameter_list:
        params = [prog._params[p] if isinstance(p, str) else p for p in parameter_list]
    _, p_grads = _build_backward(prog, [loss], no_grad_set=no_grad_set, params=params,
                                 loss_scale=loss_scale, checkpoints=checkpoints,
                                 segments_fn=segments_fn)
    if checkpoints:
        prog.__dict__['_recompute_checkpoints'] = [c.name for c in checkpoints]
    out = []
    for name, gvid in p_grads.items():
        if gvid is None:
            continue
        p = prog._params[name]
        g = blk.vars[gvid]
        g.name = name + '@GRAD'
        g.__dict__['param'] = p
        out.append((p, g))
    prog.__dict__['_param_grads'] = {id(p): g for p, g in out}
    return out


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    targets = targets if isinstance(targets, (list, tuple)) else [targets]
    inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    prog = default_main_program()
    blk = prog.global_block()
    tg = None if target_gradients is None else (
        target_gradients if isinstance(target_gradients, (list, tuple)) else [target_gradients])
    in_grads, _ = _build_backward(prog, list(targets), inputs=list(inputs), target_grads=tg,
                                  no_grad_set=no_grad_set, params=[])
    outs = []
    for x in inputs:
        gv = in_grads.get(x.vid)
        if gv is None:  # no path: a zeros op keeps the fetch valid
            g = _new_var(blk, x.shape, x.dtype, x.name + '@GRAD')
            blk.ops.append(OpDesc('fill_grad_seed', _seed, [_VarRef(x.vid), 0.0], {}, [x.vid],
                                  [g.vid], 'T', role='backward'))
            outs.append(g)
        else:
            outs.append(blk.vars[gv])
    prog._bump()
    return outs


def _optimize_fn(opt, params, *grads, scaler=None):
    """Apply ``param@GRAD`` vars through the eager optimizer (fused multi-tensor kernels)."""
    for p, g in zip(params, grads):
        gt = _u(g)
        p._t.grad = gt.to(p._t.dtype) if gt.dtype != p._t.dtype else gt
    if scaler is not None:
        scaler.step(opt)
        scaler.update()
    else:
        opt.step()
    opt.clear_grad(set_to_zero=False)
    return None


register_static_op('optimize', _optimize_fn)


def _static_minimize(opt, loss, parameters=None, scaler=None, loss_scale=1.0, checkpoints=None):
    """Backward + optimize op for ``loss``'s program. Settings recorded on the program by
    ``paddle.distributed.passes`` (``prog._pass_cfg``: amp, recompute checkpoints, gradient
    merge, sharding stage 1, gradient bucket size) are honoured here; the arguments are kept so
    a pass applied AFTER minimize can strip the training ops and rebuild them."""
    prog = loss.block.program
    check_single_device(prog)
    args = dict(opt=opt, loss=loss, parameters=parameters, scaler=scaler, loss_scale=loss_scale,
                checkpoints=checkpoints)
    cfg = prog.__dict__.get('_pass_cfg') or {}
    blk = prog.global_block()
    segments_fn = None
    if checkpoints is None and cfg.get('checkpoints'):
        checkpoints = [blk.var(c) if isinstance(c, str) else c for c in cfg['checkpoints']]
    elif checkpoints is None and cfg.get('recompute_annotated') is not None:
        skip = list(cfg['recompute_annotated'])
        segments_fn = lambda fwd: annotated_segments(fwd, skip)  # noqa: E731
    amp = cfg.get('amp')
    if amp is not None:
        from .amp import tag_program, _ScaleRef
        tag_program(prog, amp)
        if scaler is None and amp.get('scaler') is not None:
            scaler, loss_scale = amp['scaler'], _ScaleRef(amp['scaler'])
        if amp.get('level') == 'O2':
            opt._multi_precision = True
    if not opt._parameter_list:
        ps = parameters or [p for p in prog.all_parameters() if not p.stop_gradient]
        opt._param_groups = []
        opt._add_param_group({'params': list(ps)})
    groups = save_param_groups(opt)
    fwd_vids = set(blk.vars)
    n_before = len(blk.ops)
    pg = append_backward(loss, parameters, loss_scale=loss_scale, checkpoints=checkpoints,
                         segments_fn=segments_fn)
    params = [p for p, _ in pg]
    gvars = [g for _, g in pg]
    prog.__dict__['_minimize_params'] = list(params)
    sync = prog.__dict__.get('_ap_grad_sync')
    k_steps, avg = cfg.get('gradient_merge', (1, True))
    shard = cfg.get('sharding')
    if sync or k_steps > 1 or shard is not None:
        # auto-parallel partitioned program: bucketed async gradient all-reduce over the mesh
        # axes the parameters are replicated on (static_passes.Partitioner records them), the
        # merge window and the stage-1 owner update + broadcast (meta_optimizers)
        from ..distributed.fleet.meta_optimizers import build_sync_optimize
        build_sync_optimize(prog, n_before, pg, opt, scaler, sync, k_steps, avg, shard,
                            cfg.get('bucket_mb', prog.__dict__.get('_ap_bucket_mb', 32)))
    else:
        op = OpDesc('optimize', _optimize_fn, [opt, params] + [_VarRef(g.vid) for g in gvars],
                    {'scaler': scaler}, [g.vid for g in gvars], [], 'C', role='optimize')
        blk.ops.append(op)
    for hook in cfg.get('minimize_hooks', ()):
        hook(prog, opt)
    prog.__dict__['_train_meta'] = {'fwd_vids': fwd_vids, 'kind': 'plain',
                                    'rebuild': lambda: (restore_param_groups(opt, groups),
                                                        _static_minimize(**args))}
    prog._bump()
    return None, pg


def _inner_opt(opt):
    while '_optimizer' in getattr(opt, '__dict__', {}):
        opt = opt.__dict__['_optimizer']
    return opt


def save_param_groups(opt):
    """The optimizer's parameter groups as minimize saw them (sharding later narrows them to the
    owned parameters; a rebuild restores them first)."""
    return [dict(g, params=list(g['params'])) for g in _inner_opt(opt)._param_groups]


def restore_param_groups(opt, groups):
    o = _inner_opt(opt)
    o._param_groups = [dict(g, params=list(g['params'])) for g in groups]
    o._fused_plan = None


def strip_training(prog):
    """Undo append_backward / minimize: drop the grad, recompute, communication and optimize ops,
    the RNG snapshots, the forward ops' autograd-context links and the vars only those ops made.
    The program is its forward again (``_train_meta['rebuild']`` re-creates the training ops)."""
    blk = prog.global_block()
    meta = prog.__dict__.get('_train_meta') or {}
    keep = [op for op in blk.ops if op.role == 'forward' and op.type != 'recompute_rng_save']
    for op in keep:
        op.ctx_vid = None
        op.attrs.pop('diff_in', None)
        op.attrs.pop('diff_params', None)
    blk.ops[:] = keep
    fwd_vids = meta.get('fwd_vids')
    if fwd_vids is not None:
        for vid in [v for v in blk.vars if v not in fwd_vids]:
            del blk.vars[vid]
    for k in ('_param_grads', '_recompute_checkpoints', '_fleet_state', '_ap_grad_states',
              '_no_graph', '_train_meta'):
        prog.__dict__.pop(k, None)
    prog._plans = {}
    prog._bump()


def rebuild_training(prog):
    """Re-run the program's minimize (after a pass changed ``_pass_cfg``). False when the program
    has no training ops yet (the settings then apply at its minimize)."""
    meta = prog.__dict__.get('_train_meta')
    if meta is None:
        return False
    rebuild = meta['rebuild']
    strip_training(prog)
    rebuild()
    return True


class RecomputeOptimizer:
    """Static-graph activation recomputation around an inner optimizer (parity:
    python/paddle/fluid/optimizer.py:6447 RecomputeOptimizer; fleet meta_optimizers/
    recompute_optimizer.py:97). ``_set_checkpoints`` names the Variables kept in memory; the
    backward re-runs the forward ops between consecutive checkpoints (see _recompute_segments)."""

    def __init__(self, optimizer):
        from . import _static_mode_enabled
        if not _static_mode_enabled():
            raise Exception("In dygraph, don't support RecomputeOptimizer.")
        self._optimizer = optimizer
        self._checkpoints = None
        self._learning_rate = getattr(optimizer, '_learning_rate', None)

    def _set_checkpoints(self, checkpoints):
        if not isinstance(checkpoints, (list, tuple)):
            raise TypeError("_checkpoints should be a list of Variable or a list of String")
        for c in checkpoints:
            if not isinstance(c, (Variable, str)):
                raise TypeError("_checkpoints should be a list of Variable or a list of String")
        self._checkpoints = list(checkpoints)

    def _resolve(self, prog):
        if not self._checkpoints:
            raise ValueError("RecomputeOptimizer: call _set_checkpoints() before minimize/backward")
        blk = prog.global_block()
        return [blk.var(c) if isinstance(c, str) else c for c in self._checkpoints]

    def load(self, state_dict):
        raise NotImplementedError("load function is not supported by Recompute Optimizer for now")

    def backward(self, loss, startup_program=None, parameter_list=None, no_grad_set=None,
                 callbacks=None):
        return append_backward(loss, parameter_list, no_grad_set,
                               checkpoints=self._resolve(loss.block.program))

    def apply_gradients(self, params_grads):
        prog = params_grads[0][1].block.program if params_grads else default_main_program()
        opt = self._optimizer
        params = [p for p, _ in params_grads]
        if not opt._parameter_list:
            opt._param_groups = []
            opt._add_param_group({'params': list(params)})
        blk = prog.global_block()
        gvars = [g for _, g in params_grads]
        blk.ops.append(OpDesc('optimize', _optimize_fn, [opt, params] + [_VarRef(g.vid) for g in gvars],
                              {'scaler': None}, [g.vid for g in gvars], [], 'C', role='optimize'))
        prog._bump()
        return []

    def apply_optimize(self, loss, startup_program, params_grads):
        return self.apply_gradients(params_grads)

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from .amp import OptimizerWithMixedPrecision, _ScaleRef
        opt, scaler, ls = self._optimizer, None, 1.0
        ckpts = self._resolve(loss.block.program)
        if isinstance(opt, OptimizerWithMixedPrecision):
            opt._tag_program(loss.block.program)
            if opt._use_scaling:
                scaler, ls = opt._scaler, _ScaleRef(opt._scaler)
            opt = opt._optimizer
        return _static_minimize(opt, loss, parameter_list, scaler=scaler, loss_scale=ls,
                                checkpoints=ckpts)

    def __getattr__(self, k):
        return getattr(self.__dict__['_optimizer'], k)


def _tensor_bytes(t, seen):
    if not isinstance(t, torch.Tensor) or t.device.type == 'meta':
        return 0
    try:
        key = (t.untyped_storage().data_ptr(), t.device)
        n = t.untyped_storage().nbytes()
    except Exception:
        return 0
    if key in seen or not n:
        return 0
    seen.add(key)
    return n


def _live_bytes(env):
    """Bytes held by an executor environment: tensors plus what op contexts keep for the
    backward (a generic context's leaf inputs and outputs, a direct-grad context's saved
    tensors), each storage counted once."""
    seen, total = set(), 0
    for v in list(env.values()):
        if isinstance(v, Tensor):
            total += _tensor_bytes(v._t, seen)
        elif isinstance(v, _Ctx):
            for t in list(v.leaves) + list(v.outs):
                total += _tensor_bytes(t, seen)
        elif isinstance(v, _FnCtx):
            for t in v.saved_tensors:
                total += _tensor_bytes(t, seen)
    return total


# =============================================================================
# Executor
# =============================================================================
class Scope:
    def __init__(self):
        self.vars = {}

    def var(self, name):
        return self.vars.setdefault(name, None)

    def find_var(self, name):
        return self.vars.get(name)


_global_scope = Scope()


def global_scope():
    return _global_scope


@contextlib.contextmanager
def scope_guard(scope):
    global _global_scope
    prev = _global_scope
    _global_scope = scope
    try:
        yield
    finally:
        _global_scope = prev


class BuildStrategy:
    def __init__(self):
        self.use_hip_graph = False
        self.fuse_elewise_add_act_ops = False
        self.fuse_bn_act_ops = False
        self.enable_inplace = True
        self.memory_optimize = True
        self.enable_addto = False


class ExecutionStrategy:
    def __init__(self):
        self.num_threads = 1
        self.num_iteration_per_drop_scope = 1


class CompiledProgram:
    def __init__(self, program_or_graph, build_strategy=None):
        self._program = program_or_graph
        self._build_strategy = build_strategy or BuildStrategy()

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None,
                           share_vars_from=None, places=None):
        if build_strategy is not None:
            self._build_strategy = build_strategy
        return self


def _as_tensor_feed(v, var):
    if isinstance(v, Tensor):
        t = v._t
    else:
        t = torch.as_tensor(np.asarray(v))
    if var is not None and t.dtype != var.dtype:
        t = t.to(var.dtype)
    dev = _default_device()
    if t.device != dev:
        t = t.to(dev, non_blocking=True)
    if var is not None and not var.stop_gradient and t.is_floating_point():
        t = t.detach().requires_grad_()
    return Tensor(t)


class Executor:
    """Replays a Program through the kernel registry using the native scheduler's plan."""

    def __init__(self, place=None):
        self.place = place
        self._op_costs = None  # list of (op type, ms) when per-op timing is on (CostModel)
        self._mem_trace = None  # peak bytes held by the run's environment (enable_memory_trace)

    def enable_memory_trace(self, on=True):
        """Track the peak bytes the executor's environment holds during ``run`` (activations
        and backward contexts; parameters excluded): ``peak_live_bytes``."""
        self._mem_trace = 0 if on else None

    @property
    def peak_live_bytes(self):
        return self._mem_trace or 0

    def enable_op_timing(self, on=True):
        """Record every executed op's wall time (device-synchronized) in ``op_costs``."""
        self._op_costs = [] if on else None

    @property
    def op_costs(self):
        return list(self._op_costs or [])

    def close(self):
        pass

    def _plan(self, prog, required):
        key = (prog._version, tuple(required))
        plan = prog._plans.get(key)
        if plan is None:
            from ..native import build_plan
            ops = prog.global_block().ops
            ins = [op.in_vids for op in ops]
            outs = [op.all_outputs() for op in ops]
            persist = [v.vid for v in prog.global_block().vars.values() if v.persistable]
            order, free_after, level, pruned = build_plan(ins, outs, list(required), persist)
            plan = (order, free_after)
            prog._plans[key] = plan
        return plan

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name='feed',
            fetch_var_name='fetch', scope=None, return_numpy=True, use_program_cache=True,
            use_prune=False):
        use_graph = False
        if isinstance(program, CompiledProgram):
            use_graph = program._build_strategy.use_hip_graph
            program = program._program
        prog = program or default_main_program()
        if prog.__dict__.get('_pipeline') is not None:
            # a pipeline stage (static/pipeline.py): micro-batched schedule with p2p transfers
            return prog._pipeline.run(self, feed or {}, list(fetch_list or []), return_numpy)
        if prog.__dict__.get('_no_graph'):
            use_graph = False   # fleet collective programs (meta_optimizers.static_minimize)
        if prog._is_startup or not prog.global_block().ops and not fetch_list:
            return []
        feed = feed or {}
        fetch_list = list(fetch_list or [])
        blk = prog.global_block()
        fetch_vars = []
        for f in fetch_list:
            if isinstance(f, str):
                f = blk.var(f) if blk.has_var(f) else prog._params[f]
            fetch_vars.append(f)
        names = list(feed.keys())
        vals = [_as_tensor_feed(feed[n], blk.var(n)) for n in names]
        has_opt = any(op.role == 'optimize' for op in blk.ops)
        if use_graph and torch.cuda.is_available() and vals and all(v._t.is_cuda for v in vals):
            from ..jit.api import _GraphEntry, _signature
            key = (prog._version, tuple(names), _signature(tuple(vals), {}),
                   tuple(id(f) for f in fetch_vars))
            cache = prog.__dict__.setdefault('_graph_cache', {})
            g = cache.get(key)
            opt_ops = [op for op in blk.ops if op.role == 'optimize']
            opt_in = [blk.vars[v] for op in opt_ops for v in op.in_vids]
            nf = len(fetch_vars)
            if g is None:
                # forward + backward (grad ops) captured as ONE HIP graph; the optimizer
                # step (host-side LR / loss-scale state) runs eagerly after each replay
                fn = lambda *fv: self._execute(prog, names, fv, fetch_vars + opt_in,  # noqa: E731
                                               skip_optimize=True)
                if has_opt:
                    g = cache[key] = _GraphEntry(fn, tuple(vals), {})
                else:
                    with torch.no_grad():
                        g = cache[key] = _GraphEntry(fn, tuple(vals), {})
            # static buffers: the fetches are copied out here, the gradients feed the optimizer
            # ops below before the next replay (no per-step clone of every gradient)
            res = g.replay_static(tuple(vals), {})
            outs = [Tensor(o._t.clone()) for o in res[:nf]]
            if opt_ops:
                genv = {v.vid: t for v, t in zip(opt_in, res[nf:])}
                prev = _STATIC[0]
                _STATIC[0] = False
                try:
                    for op in opt_ops:
                        op.fn(*_materialize(op.args, genv), **_materialize(op.kwargs, genv))
                finally:
                    _STATIC[0] = prev
        else:
            outs = self._execute(prog, names, vals, fetch_vars)
        return [t.numpy() if return_numpy else t for t in outs]

    def _run_op(self, op, env, ctx_needed, explicit_bwd):
        amp_cfg = op.attrs.get('amp')
        amp_ctx = contextlib.nullcontext()
        if amp_cfg is not None:
            from ..amp import auto_cast
            amp_ctx = auto_cast(True, amp_cfg['white'], amp_cfg['black'], amp_cfg['level'],
                                amp_cfg['dtype'])
        with amp_ctx:
            if op.role in _FWD_ROLES and op.ctx_vid is not None and ctx_needed and \
                    op.type in _FN_OPS and not op.kwargs:
                r = self._run_fn_op(op, env)
                if r is not None:
                    return r
            if op.role in _FWD_ROLES and op.ctx_vid is not None and ctx_needed:
                # run on leaf copies of the differentiable inputs and keep this op's own graph
                diff_in = op.attrs.get('diff_in', [])
                dps = op.attrs.get('diff_params', [])
                overlay = {}
                for vid in diff_in:
                    t = _u(env[vid]).detach()
                    if t.is_floating_point() or t.is_complex():
                        t.requires_grad_(True)
                    overlay[vid] = Tensor(t)
                view = collections.ChainMap(overlay, env)
                with torch.enable_grad():
                    res = op.fn(*_materialize(op.args, view), **_materialize(op.kwargs, view))
                flat, _ = _flatten_out(res)
                env[op.ctx_vid] = _Ctx([overlay[v]._t for v in diff_in], [p._t for p in dps],
                                       [t._t for t in flat])
                return [Tensor(t._t.detach()) for t in flat]
            if op.role == 'optimize' or not explicit_bwd:
                # programs without grad ops (inference, TranslatedLayer fine-tuning) keep the
                # ambient autograd mode so eager backward can flow through them
                return op.fn(*_materialize(op.args, env), **_materialize(op.kwargs, env))
            with torch.no_grad():
                return op.fn(*_materialize(op.args, env), **_materialize(op.kwargs, env))

    def _run_fn_op(self, op, env):
        """Forward of a direct-grad op: Function.forward on a _FnCtx (None: predicate declined)."""
        if not _DIRECT_GRAD:
            return None
        fn_cls, pred = _FN_OPS[op.type]
        vals = _materialize(op.args, env)
        targs = [_u(a) if isinstance(a, Tensor) else a for a in vals]
        nfwd = fn_cls.__dict__.get('_pra_nargs')
        if nfwd is None:
            nfwd = len(inspect.signature(fn_cls.forward).parameters) - 1
            setattr(fn_cls, '_pra_nargs', nfwd)
        targs += [None] * (nfwd - len(targs))  # trailing optional args left at None (e.g. bias)
        if pred is not None and not pred(*targs):
            return None
        diff_in = op.attrs.get('diff_in', [])
        dps = op.attrs.get('diff_params', [])
        slots, needs = [], []
        for a in op.args:
            if isinstance(a, _VarRef):
                key = ('v', a.vid)
                slots.append(key)
                needs.append(a.vid in diff_in)
            elif isinstance(a, Tensor) and any(a is p for p in dps):
                key = ('p', id(a))
                slots.append(key)
                needs.append(True)
            else:
                slots.append(None)
                needs.append(False)
        order = [('v', v) for v in diff_in] + [('p', id(p)) for p in dps]
        ctx = _FnCtx(fn_cls, tuple(needs), slots, order)
        with torch.no_grad():
            out = fn_cls.forward(ctx, *targs)
        outs = out if isinstance(out, tuple) else (out,)
        ctx.out_meta = [(o.shape, o.dtype, o.device) for o in outs]
        env[op.ctx_vid] = ctx
        return tuple(Tensor(o) for o in outs) if isinstance(out, tuple) else Tensor(out)

    def _execute(self, prog, names, vals, fetch_vars, skip_optimize=False):
        blk = prog.global_block()
        required = [f.vid for f in fetch_vars if isinstance(f, Variable) and
                    not isinstance(f, GradVar)]
        order, free_after = self._plan(prog, required)
        env = {blk.var(n).vid: v for n, v in zip(names, vals)}
        prev = _STATIC[0]
        _STATIC[0] = False
        try:
            ops = blk.ops
            live = {v for oi in order for v in ops[oi].in_vids}
            explicit_bwd = any(ops[oi].role in ('backward', 'recompute') for oi in order)
            timing = self._op_costs is not None
            sync = torch.cuda.synchronize if timing and torch.cuda.is_available() else \
                (lambda: None)
            for pos, oi in enumerate(order):
                op = ops[oi]
                if skip_optimize and op.role == 'optimize':
                    continue
                if timing:
                    sync()
                    t0 = time.perf_counter()
                res = self._run_op(op, env, op.ctx_vid in live, explicit_bwd)
                if timing:
                    sync()
                    self._op_costs.append((op.type, (time.perf_counter() - t0) * 1e3))
                if op.out_vids:
                    if isinstance(res, list) and len(res) == len(op.out_vids) and any(r is None for r in res):
                        flat = res   # an op that produced no value for some outputs this run
                    else:
                        flat, _ = _flatten_out(res)
                    for vid, t in zip(op.out_vids, flat):
                        env[vid] = t
                if self._mem_trace is not None:
                    self._mem_trace = max(self._mem_trace, _live_bytes(env))
                for vid in free_after[pos]:
                    if vid not in required:
                        env.pop(vid, None)
        finally:
            _STATIC[0] = prev
        results = []
        for f in fetch_vars:
            if isinstance(f, GradVar):
                g = f.param._t.grad
                t = Tensor(g if g is not None else torch.zeros_like(f.param._t))
            elif isinstance(f, Variable):
                t = env[f.vid]
            else:
                t = f
            results.append(t)
        return results


# =============================================================================
# inference model save / load (.pdmodel ProgramDesc protobuf + .pdiparams)
# =============================================================================
def _qualname(fn, op_type=None):
    if op_type and ':' in op_type and not op_type.startswith('layer:'):
        return op_type
    if op_type and op_type.startswith('layer:'):
        raise TypeError(f"op '{op_type}' wraps a Layer whose forward is not built from paddle "
                        "ops; it can run in a Program but cannot be serialized")
    f = getattr(fn, '__wrapped__', fn)
    return f'{f.__module__}:{f.__qualname__}'


_NOT_LOADABLE = {'py_func', 'Print'}


def _resolve(op_type):
    """A .pdmodel names ops ONLY by registered op type (the static op table filled by
    ``install_static_hooks``); anything else -- e.g. a crafted 'os:system' -- is refused
    instead of being imported (parity: OpDesc.type resolved through the OpInfoMap)."""
    install_static_hooks()
    fn = _OP_TABLE.get(op_type)
    if fn is None or op_type in _NOT_LOADABLE:
        raise ValueError(f"op type {op_type!r} is not a registered paddle_ray_amd op; refusing "
                         "to load this program")
    return fn


class _LoadedBlock:
    """A control-flow sub-block read back from a ``.pdmodel`` (the serialized twin of
    control_flow._SubBlock): its ops, the vids of its placeholders / captured outer variables,
    and its output structure. ``run`` interprets it like the traced original."""
    _pra_block = True

    def __init__(self, ops, ph_vids, cap_vids, outputs):
        self.ops, self.ph_vids, self.cap_vids, self.outputs = ops, ph_vids, cap_vids, outputs

    def block_ops(self):
        return self.ops

    def run(self, feed_vals, captured_vals, out_obj=None):
        env = dict(zip(self.ph_vids, feed_vals))
        env.update(zip(self.cap_vids, captured_vals))
        return run_block_ops(self.ops, env, self.outputs if out_obj is None else out_obj)


def run_block_ops(ops, env, outputs):
    """Interpret ``ops`` over ``env`` (vid -> tensor) and resolve ``outputs`` from it."""
    for op in ops:
        res = op.fn(*_materialize(op.args, env), **_materialize(op.kwargs, env))
        if op.out_vids:
            flat, _ = _flatten_out(res)
            for vid, t in zip(op.out_vids, flat):
                env[vid] = t
    return _resolve_refs(outputs, env)


def _resolve_refs(obj, env):
    if isinstance(obj, (Variable, _VarRef)):
        return env[obj.vid]
    if isinstance(obj, (list, tuple)):
        return type(obj)(_resolve_refs(o, env) for o in obj)
    return obj


def _as_refs(obj):
    if isinstance(obj, Variable):
        return _VarRef(obj.vid)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_as_refs(o) for o in obj)
    return obj


def _encode_ops(ops, params):
    enc = []
    for op in ops:
        qn = _qualname(op.fn, op.type)
        if qn not in _OP_TABLE:
            raise TypeError(f"op {op.type!r} is not a registered static op; cannot serialize")
        enc.append({'type': qn, 'args': _encode(op.args, params),
                    'kwargs': _encode(op.kwargs, params), 'in': op.in_vids, 'out': op.out_vids})
    return enc


def _decode_ops(enc, params):
    return [OpDesc(o['type'], _resolve(o['type']), _decode(o['args'], params),
                   _decode(o['kwargs'], params), o['in'], o['out'], None) for o in enc]


def _encode(obj, params):
    if getattr(obj, '_pra_block', False):  # a control-flow sub-block: nested op list
        return {'__block__': {'ops': _encode_ops(obj.block_ops(), params),
                              'ph': list(obj.ph_vids), 'cap': list(obj.cap_vids),
                              'out': _encode(_as_refs(obj.outputs), params)}}
    if isinstance(obj, _VarRef):
        return {'__var__': obj.vid}
    if isinstance(obj, Tensor):
        if isinstance(obj, Parameter) or obj.persistable:
            params[obj.name] = obj
            return {'__param__': obj.name}
        return {'__const__': obj.numpy().tolist(), 'dtype': dtype_to_str(obj.dtype)}
    if isinstance(obj, torch.dtype):
        return {'__dtype__': dtype_to_str(obj)}
    if isinstance(obj, slice):
        return {'__slice__': [obj.start, obj.stop, obj.step]}
    if obj is Ellipsis:
        return {'__ellipsis__': 1}
    if isinstance(obj, tuple):
        return {'__tuple__': [_encode(o, params) for o in obj]}
    if isinstance(obj, list):
        return [_encode(o, params) for o in obj]
    if isinstance(obj, dict):
        return {'__dict__': {k: _encode(v, params) for k, v in obj.items()}}
    if isinstance(obj, (np.integer,)):
        return int(obj)
    if isinstance(obj, (np.floating,)):
        return float(obj)
    if obj is None or isinstance(obj, (bool, int, float, str)):
        return obj
    raise TypeError(f"cannot serialize op argument of type {type(obj)}")


def _decode(obj, params):
    if isinstance(obj, list):
        return [_decode(o, params) for o in obj]
    if isinstance(obj, dict):
        if '__var__' in obj:
            return _VarRef(obj['__var__'])
        if '__block__' in obj:
            b = obj['__block__']
            return _LoadedBlock(_decode_ops(b['ops'], params), b['ph'], b['cap'],
                                _decode(b['out'], params))
        if '__param__' in obj:
            return params[obj['__param__']]
        if '__const__' in obj:
            return Tensor(torch.as_tensor(np.asarray(obj['__const__'], dtype=obj['dtype']),
                                          device=_default_device()))
        if '__dtype__' in obj:
            return convert_dtype(obj['__dtype__'])
        if '__slice__' in obj:
            return slice(*obj['__slice__'])
        if '__ellipsis__' in obj:
            return Ellipsis
        if '__tuple__' in obj:
            return tuple(_decode(o, params) for o in obj['__tuple__'])
        if '__dict__' in obj:
            return {k: _decode(v, params) for k, v in obj['__dict__'].items()}
    return obj


def _ordered_forward_ops(blk, required):
    from ..native import build_plan
    ops = [op for op in blk.ops if op.role == 'forward']
    order, _, _, _ = build_plan([o.in_vids for o in ops], [o.out_vids for o in ops], required, [])
    return [ops[i] for i in order]


class _DescWriter:
    """Program -> ProgramDesc dict (static/program_desc.py documents the mapping)."""

    def __init__(self, blk):
        self.blk, self.names, self.taken, self.blocks = blk, {}, set(), []

    def name(self, vid):
        n = self.names.get(vid)
        if n is None:
            v = self.blk.vars.get(vid)
            v = _ALL_VARS.get(vid) if v is None else v
            n = v.name if v is not None and v.name else f'_pra_var_{vid}'
            if n in self.taken or n in ('feed', 'fetch'):
                n = f'{n}@{vid}'
            self.names[vid] = n
            self.taken.add(n)
        return n

    def var(self, vid, params):
        from . import program_desc as PD
        v = self.blk.vars.get(vid)
        v = _ALL_VARS.get(vid) if v is None else v
        shape = v.shape if v is not None else []
        dt = dtype_to_str(v.dtype) if v is not None else 'float32'
        return PD.var_desc(self.name(vid), shape, dt, stop_gradient=bool(v is None or v.stop_gradient),
                           need_check_feed=bool(v is not None and getattr(v, 'is_data', False)))

    def _names_in(self, obj, blocks_out, parent):
        """Rewrite an _encode()d structure: var vids -> names, nested op lists -> sub-blocks."""
        if isinstance(obj, list):
            return [self._names_in(o, blocks_out, parent) for o in obj]
        if isinstance(obj, dict):
            if '__var__' in obj:
                return {'__var__': self.name(obj['__var__'])}
            if '__block__' in obj:
                b = obj['__block__']
                idx = self.block(b['ops'], parent, extra_vids=list(b['ph']) + list(b['cap']))
                blocks_out.append(idx)
                return {'__block__': {'idx': idx, 'ph': [self.name(v) for v in b['ph']],
                                      'cap': [self.name(v) for v in b['cap']],
                                      'out': self._names_in(b['out'], blocks_out, parent)}}
            return {k: self._names_in(v, blocks_out, parent) for k, v in obj.items()}
        return obj

    def op(self, enc, idx):
        from . import program_desc as PD
        subs = []
        call = {'args': self._names_in(enc['args'], subs, idx),
                'kwargs': self._names_in(enc['kwargs'], subs, idx)}
        attrs = [{'name': '__pra_call__', 'type': PD.ATTR['STRING'], 's': PD.dumps_call(call)}]
        kw = enc['kwargs'].get('__dict__', {}) if isinstance(enc['kwargs'], dict) else {}
        for k, v in sorted(kw.items()):
            a = PD.scalar_attr(k, v)
            if a is not None and not k.startswith('__'):
                attrs.append(a)
        if len(subs) == 1:
            attrs.append({'name': 'sub_block', 'type': PD.ATTR['BLOCK'], 'block_idx': subs[0]})
        elif subs:
            attrs.append({'name': 'sub_blocks', 'type': PD.ATTR['BLOCKS'], 'blocks_idx': subs})
        return {'type': enc['type'],
                'inputs': [{'parameter': 'X', 'arguments': [self.name(v) for v in enc['in']]}],
                'outputs': [{'parameter': 'Out', 'arguments': [self.name(v) for v in enc['out']]}],
                'attrs': attrs}

    def block(self, enc_ops, parent, extra_vids=(), params=None):
        idx = len(self.blocks)
        bd = {'idx': idx, 'parent_idx': parent, 'vars': [], 'ops': []}
        self.blocks.append(bd)
        bd['ops'] = [self.op(o, idx) for o in enc_ops]
        vids = list(extra_vids)
        for o in enc_ops:
            vids += list(o['in']) + list(o['out'])
        for vid in dict.fromkeys(vids):
            if idx == 0 or vid not in self.blk.vars:
                bd['vars'].append(self.var(vid, params))
        return idx


def serialize_program(feed_vars, fetch_vars, program=None):
    """ProgramDesc protobuf bytes of the forward ops reaching ``fetch_vars`` (parity:
    static/io.py serialize_program -> framework.proto ProgramDesc)."""
    from . import program_desc as PD
    prog = program or default_main_program()
    blk = prog.global_block()
    required = [v.vid for v in fetch_vars]
    params = {}
    enc_ops = _encode_ops(_ordered_forward_ops(blk, required), params)
    w = _DescWriter(blk)
    w.block(enc_ops, -1, extra_vids=[v.vid for v in feed_vars] + required)
    b0 = w.blocks[0]
    b0['vars'] = [vd for vd in b0['vars']]
    b0['vars'].insert(0, {'name': 'feed', 'persistable': True,
                          'type': {'type': PD.VT_FEED_MINIBATCH}})
    b0['vars'].insert(1, {'name': 'fetch', 'persistable': True, 'type': {'type': PD.VT_FETCH_LIST}})
    for name, p in sorted(params.items()):
        b0['vars'].append(PD.var_desc(name, list(p.shape), dtype_to_str(p.dtype), persistable=True,
                                      is_parameter=True, stop_gradient=p.stop_gradient))
    feeds = [{'type': 'feed', 'inputs': [{'parameter': 'X', 'arguments': ['feed']}],
              'outputs': [{'parameter': 'Out', 'arguments': [w.name(v.vid)]}],
              'attrs': [{'name': 'col', 'type': PD.ATTR['INT'], 'i': i}]}
             for i, v in enumerate(feed_vars)]
    fetches = [{'type': 'fetch', 'inputs': [{'parameter': 'X', 'arguments': [w.name(vid)]}],
                'outputs': [{'parameter': 'Out', 'arguments': ['fetch']}],
                'attrs': [{'name': 'col', 'type': PD.ATTR['INT'], 'i': i}]}
               for i, vid in enumerate(required)]
    b0['ops'] = feeds + b0['ops'] + fetches
    desc = {'blocks': w.blocks, 'version': {'version': PD.PROGRAM_VERSION}}
    return PD.encode('ProgramDesc', desc), params


def serialize_persistables(feed_vars, fetch_vars, executor=None, program=None):
    _, params = serialize_program(feed_vars, fetch_vars, program)
    import io
    from ..framework.io import save
    buf = io.BytesIO()
    save({k: v for k, v in params.items()}, buf)
    return buf.getvalue()


def save_inference_model(path_prefix, feed_vars, fetch_vars, executor=None, program=None,
                         **kwargs):
    feed_vars = feed_vars if isinstance(feed_vars, (list, tuple)) else [feed_vars]
    fetch_vars = fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars]
    desc, params = serialize_program(feed_vars, fetch_vars, program)
    d = os.path.dirname(path_prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path_prefix + '.pdmodel', 'wb') as f:
        f.write(desc)
    from ..framework.io import save
    save(params, path_prefix + '.pdiparams')


def _deserialize_json(data, params=None):
    """The round-1/2 JSON op-list .pdmodel (still readable)."""
    desc = json.loads(data.decode() if isinstance(data, bytes) else data)
    prog = Program()
    blk = prog.global_block()
    vmap = {}
    for vid, info in desc['vars'].items():
        v = Variable(blk, info['shape'], info['dtype'], name=info['name'],
                     is_data=int(vid) in desc['feeds'])
        vmap[int(vid)] = v
    params = params or {}
    for vid, v in vmap.items():
        v.__dict__['vid'] = vid
        blk.vars[vid] = v
    for p in params.values():
        prog._register_param(p)
    for o in desc['ops']:
        fn = _resolve(o['type'])
        op = OpDesc(o['type'], fn, _decode(o['args'], params), _decode(o['kwargs'], params),
                    o['in'], o['out'], None)
        blk.ops.append(op)
    prog._feeds = [vmap[i] for i in desc['feeds']]
    prog._fetches = [vmap[i] for i in desc['fetches']]
    prog._bump()
    return prog


def deserialize_program(data, params=None):
    """Program from ProgramDesc protobuf bytes (or a legacy JSON .pdmodel). Ops are rebuilt
    ONLY from registered op types (``_resolve``); parameters bind by name to ``params``."""
    from . import program_desc as PD
    if not PD.is_program_desc(data):
        return _deserialize_json(data, params)
    desc = PD.decode('ProgramDesc', bytes(data))
    blocks = desc.get('blocks', [])
    if not blocks:
        raise ValueError("ProgramDesc has no blocks")
    params = params or {}
    prog = Program()
    blk = prog.global_block()
    vids = {}
    feeds, fetches = {}, {}
    for b in blocks:
        for vd in b.get('vars', []):
            name, shape, dt = PD.var_info(vd)
            if dt is None or name in params or name in vids:
                continue
            v = Variable(blk, shape, dt, name=name, is_data=bool(vd.get('need_check_feed')))
            vids[name] = v.vid
            if b.get('idx', 0) == 0:
                blk.vars[v.vid] = v
            else:
                blk.__dict__.setdefault('_sub_vars', []).append(v)  # keep them alive
    for p in params.values():
        prog._register_param(p)

    def names_to_vids(obj):
        if isinstance(obj, list):
            return [names_to_vids(o) for o in obj]
        if isinstance(obj, dict):
            if '__var__' in obj:
                return {'__var__': vids[obj['__var__']]}
            if '__block__' in obj:
                b = obj['__block__']
                return {'__block__': {'ops': enc_block(b['idx']),
                                      'ph': [vids[n] for n in b['ph']],
                                      'cap': [vids[n] for n in b['cap']],
                                      'out': names_to_vids(b['out'])}}
            return {k: names_to_vids(v) for k, v in obj.items()}
        return obj

    def enc_op(od):
        attrs = {a['name']: a for a in od.get('attrs', [])}
        call = attrs.get('__pra_call__')
        if call is None:
            raise ValueError(f"op {od.get('type')!r} carries no __pra_call__ attribute: not a "
                             "paddle_ray_amd program")
        c = PD.loads_call(PD.attr_value(call))
        slot = lambda vs: [vids[n] for s in vs for n in s.get('arguments', [])]  # noqa: E731
        return {'type': od['type'], 'args': names_to_vids(c['args']),
                'kwargs': names_to_vids(c['kwargs']), 'in': slot(od.get('inputs', [])),
                'out': slot(od.get('outputs', []))}

    def enc_block(idx):
        return [enc_op(od) for od in blocks[idx].get('ops', [])]

    mixed = None
    for od in blocks[0].get('ops', []):
        attrs = {a['name']: a for a in od.get('attrs', [])}
        if od['type'] == MIXED_PRECISION_OP:
            mixed = json.loads(PD.attr_value(attrs['config']))
            continue
        if od['type'] == 'feed':
            feeds[PD.attr_value(attrs['col'])] = od['outputs'][0]['arguments'][0]
            continue
        if od['type'] == 'fetch':
            fetches[PD.attr_value(attrs['col'])] = od['inputs'][0]['arguments'][0]
            continue
        o = enc_op(od)
        blk.ops.append(OpDesc(o['type'], _resolve(o['type']), _decode(o['args'], params),
                              _decode(o['kwargs'], params), o['in'], o['out'], None))
    prog._feeds = [blk.vars[vids[feeds[i]]] for i in sorted(feeds)]
    for v in prog._feeds:
        v.__dict__['is_data'] = True
    prog._fetches = [blk.vars[vids[fetches[i]]] for i in sorted(fetches)]
    if mixed is not None:
        apply_mixed_precision(prog, mixed)
    prog._bump()
    return prog


# A converted mixed-precision model (inference.convert_to_mixed_precision) carries one marker op
# of this type in block 0 with a STRING attribute 'config' = {"dtype", "black_list",
# "keep_io_types"}: on load every op replays under O2 autocast of that dtype, black-listed op
# types in fp32.
MIXED_PRECISION_OP = 'pra_mixed_precision'


def apply_mixed_precision(prog, cfg):
    from ..amp import BLACK_LIST
    dt = {'float16': torch.float16, 'bfloat16': torch.bfloat16}[cfg['dtype']]
    black = set(cfg.get('black_list', [])) | set(BLACK_LIST)
    amp = {'dtype': dt, 'level': 'O2', 'white': set(), 'black': black}
    for op in prog.global_block().ops:
        if op.type in set(cfg.get('black_list', [])):
            continue
        op.attrs['amp'] = amp
    prog.__dict__['_mixed_precision'] = dict(cfg)


def load_inference_model(path_prefix, executor=None, **kwargs):
    from ..framework.io import load
    raw = load(path_prefix + '.pdiparams')
    params = {}
    for k, v in raw.items():
        p = Parameter(v._t.to(_default_device()), trainable=False, name=k)
        params[k] = p
    with open(path_prefix + '.pdmodel', 'rb') as f:
        prog = deserialize_program(f.read(), params)
    return [prog, [v.name for v in prog._feeds], prog._fetches]


def save(program, model_path, protocol=4, **configs):
    from ..framework.io import save as _save
    _save(program.state_dict(), model_path + '.pdparams')


def load(program, model_path, executor=None, var_list=None):
    from ..framework.io import load as _load
    program.set_state_dict(_load(model_path + '.pdparams'))


def load_program_state(model_path, var_list=None):
    from ..framework.io import load as _load
    return {k: v.numpy() for k, v in _load(model_path + '.pdparams').items()}


def set_program_state(program, state_dict):
    program.set_state_dict(state_dict)


def normalize_program(program, feed_vars, fetch_vars):
    return program.clone(for_test=True)


def save_to_file(path, content):
    with open(path, 'wb') as f:
        f.write(content)


def load_from_file(path):
    with open(path, 'rb') as f:
        return f.read()


def deserialize_persistables(program, data, executor=None):
    import io
    from ..framework.io import load as _load
    program.set_state_dict(_load(io.BytesIO(data)))


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..tensor.creation import create_parameter as cp
    p = cp(shape, dtype, name, attr, is_bias, default_initializer)
    default_main_program()._register_param(p)
    return p


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    from ..tensor.creation import full
    t = full(shape, value, dtype)
    t.persistable = True
    t.name = name or t.name
    return t


def _print_fn(x, message=''):
    print(message, x)
    return x


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True,
          print_tensor_type=True, print_tensor_shape=True, print_tensor_lod=True,
          print_phase='both'):
    return static_op('Print', _print_fn)(input, message or '')


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    def run(*a):
        return func(*a)
    if _STATIC[0] and _has_var(xs):
        return record_op('py_func', run, xs, {})  # runs in-process; never serialized
    return run(*xs)


def cpu_places(device_count=None):
    from ..framework.core import CPUPlace
    return [CPUPlace()] * (device_count or 1)


def cuda_places(device_ids=None):
    from ..framework.core import CUDAPlace
    ids = device_ids if device_ids is not None else range(max(torch.cuda.device_count(), 1))
    return [CUDAPlace(i) for i in ids]


def xpu_places(device_ids=None):
    return []


npu_places = mlu_places = xpu_places


def accuracy(input, label, k=1, correct=None, total=None):
    from ..metric import accuracy as acc
    return static_op('accuracy', acc)(input, label, k)


def _stateful_metric(name, fn, args, specs):
    """Run ``fn`` now (eager) or record it as one op whose persistable state lives in ``fn``'s
    closure and is updated every time the program executes (``out_specs`` given, so shape
    inference never runs the update on probe data)."""
    if _STATIC[0] and _has_var(args):
        flat = [(list(s), d) for s, d in specs]
        tmpl = ('tuple', ['T'] * len(flat))
        return record_op(name, fn, list(args), {}, out_specs=(tmpl, flat))
    return fn(*args)


def auc(input, label, curve='ROC', num_thresholds=4095, topk=1, slide_steps=1,
        ins_tag_weight=None):
    """Streaming AUC over bucketed positive-class scores (parity: python/paddle/static/nn/
    metric.py auc). Returns (auc, batch_auc, [batch_stat_pos, batch_stat_neg, stat_pos,
    stat_neg]); the global stats accumulate over every run, the batch stats over the last
    ``slide_steps`` runs (0 = all)."""
    nb = num_thresholds + 1
    st = {'pos': torch.zeros(nb, dtype=torch.float64), 'neg': torch.zeros(nb, dtype=torch.float64),
          'win': []}

    def _area(pos, neg):
        # thresholds from high to low: trapezoids of (FP, TP) (ROC) or (recall, precision) (PR)
        tp = torch.cumsum(pos.flip(0), 0)
        fp = torch.cumsum(neg.flip(0), 0)
        P, N = tp[-1], fp[-1]
        if curve.upper() == 'PR':
            prec = tp / (tp + fp).clamp(min=1)
            rec = tp / P.clamp(min=1)
            r0 = torch.cat([rec.new_zeros(1), rec[:-1]])
            p0 = torch.cat([prec.new_ones(1), prec[:-1]])
            return float(((rec - r0) * (prec + p0) / 2).sum())
        if P == 0 or N == 0:
            return 0.0
        tp0 = torch.cat([tp.new_zeros(1), tp[:-1]])
        fp0 = torch.cat([fp.new_zeros(1), fp[:-1]])
        return float(((fp - fp0) * (tp + tp0) / 2).sum() / (P * N))

    def run(pred, lab, *tw):
        p = _u(pred).detach().double().cpu()
        score = p[:, -1] if p.dim() == 2 and p.shape[1] > 1 else p.reshape(-1)
        y = _u(lab).reshape(-1).cpu() != 0
        if tw and float(_u(tw[0]).reshape(-1)[0]) == 0:
            y = y[:0]
            score = score[:0]
        bucket = (score * num_thresholds).long().clamp(0, num_thresholds)
        bp = torch.bincount(bucket[y], minlength=nb).double()
        bn = torch.bincount(bucket[~y], minlength=nb).double()
        st['pos'] += bp
        st['neg'] += bn
        st['win'].append((bp, bn))
        if slide_steps > 0:
            st['win'] = st['win'][-slide_steps:]
        wp = sum(w[0] for w in st['win'])
        wn = sum(w[1] for w in st['win'])
        dev = _u(pred).device
        f = lambda v: Tensor(torch.tensor([v], dtype=torch.float64, device=dev))  # noqa: E731
        g = lambda v: Tensor(v.to(dev).reshape(1, -1).to(torch.int64))  # noqa: E731
        return (f(_area(st['pos'], st['neg'])), f(_area(wp, wn)), g(wp), g(wn), g(st['pos']),
                g(st['neg']))

    args = [input, label] + ([ins_tag_weight] if ins_tag_weight is not None else [])
    specs = [([1], torch.float64)] * 2 + [([1, nb], torch.int64)] * 4
    out = _stateful_metric('auc', run, args, specs)
    return out[0], out[1], list(out[2:])


class WeightNormParamAttr:
    def __init__(self, dim=None, **kw):
        self.dim = dim


class ExponentialMovingAverage:
    def __init__(self, decay=0.999, thres_steps=None, name=None):
        self.decay = decay
        self._shadow = {}

    def update(self):
        for n, p in default_main_program()._params.items():
            s = self._shadow.setdefault(n, p._t.detach().clone())
            s.mul_(self.decay).add_(p._t.detach(), alpha=1 - self.decay)

    @contextlib.contextmanager
    def apply(self, executor=None, need_restore=True):
        backup = {}
        for n, p in default_main_program()._params.items():
            if n in self._shadow:
                backup[n] = p._t.detach().clone()
                p._t.data.copy_(self._shadow[n])
        yield
        if need_restore:
            for n, t in backup.items():
                default_main_program()._params[n]._t.data.copy_(t)


def ipu_shard_guard(*a, **k):
    return contextlib.nullcontext()


def set_ipu_shard(*a, **k):
    return None


class IpuStrategy:
    pass


class IpuCompiledProgram:
    pass


ParallelExecutor = Executor


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    from ..optimizer.lr import ExponentialDecay
    return ExponentialDecay(learning_rate, decay_rate ** (1.0 / decay_steps))


def ctr_metric_bundle(input, label, ins_tag_weight=None):
    """Running CTR sums (parity: python/paddle/fluid/contrib/layers/metric_op.py
    ctr_metric_bundle): squared error, absolute error, predicted-ctr sum, q (sum of
    sigmoid(input)), positives and instance count, accumulated over every run; a batch whose
    ins_tag_weight is 0 (fake data) adds nothing to q and the instance count."""
    st = torch.zeros(6, dtype=torch.float32)

    def run(pred, lab, *tw):
        p = _u(pred).detach().float().cpu().reshape(-1)
        y = _u(lab).detach().float().cpu().reshape(-1)
        w = float(_u(tw[0]).reshape(-1)[0]) if tw else 1.0
        d = p - y
        st.add_(torch.stack([(d * d).sum(), d.abs().sum(), p.sum(), torch.sigmoid(p).sum() * w,
                                 y.sum(), torch.tensor(float(p.numel())) * w]))
        dev = _u(pred).device
        return tuple(Tensor(st[i:i + 1].clone().to(dev)) for i in range(6))

    args = [input, label] + ([ins_tag_weight] if ins_tag_weight is not None else [])
    return _stateful_metric('ctr_metric_bundle', run, args, [([1], torch.float32)] * 6)


ctc_metric_bundle = ctr_metric_bundle


# =============================================================================
# Layer-level recording + hook installation
# =============================================================================
def _snapshot(prog):
    blk = prog.global_block()
    return len(blk.ops), set(blk.vars)


def _rollback(prog, snap):
    blk = prog.global_block()
    n, vids = snap
    del blk.ops[n:]
    for vid in list(blk.vars):
        if vid not in vids:
            del blk.vars[vid]
    prog._bump()


def _all_vars(out):
    flat, _ = _flatten_out(out)
    return bool(flat) and all(isinstance(t, Variable) for t in flat)


def _real_probe_env(block, probe, extra=()):
    env = {}
    dev = _default_device()
    for vid, v in _scope_vars(block, extra).items():
        shp = [probe if s < 0 else s for s in v._vshape]
        env[vid] = Tensor(torch.zeros(shp, dtype=v.dtype, device=dev))
    return env


def record_layer_call(layer, inputs, kwargs):
    """Record a Layer call: as its primitive ops when its forward is built from paddle
    ops, else (forward touches raw tensors) as ONE layer op replayed by the Executor."""
    prog = default_main_program()
    snap = _snapshot(prog)
    try:
        out = layer._call_impl(*inputs, **kwargs)
        if _all_vars(out):
            return out
    except Exception:
        pass
    _rollback(prog, snap)
    for p in layer.parameters():
        prog._register_param(p)
    blk = prog.global_block()
    in_vids, params = [], []
    targs = _template(list(inputs), in_vids, params)
    tkw = _template(dict(kwargs), in_vids, params)

    def call(*a, **k):
        return layer._call_impl(*a, **k)

    outs = []
    for probe in _PROBES:
        env = _real_probe_env(blk, probe)
        prev = _STATIC[0]
        _STATIC[0] = False
        try:
            with torch.no_grad():
                outs.append(call(*_materialize(targs, env), **_materialize(tkw, env)))
        finally:
            _STATIC[0] = prev
    flat0, tmpl = _flatten_out(outs[0])
    flat1, _ = _flatten_out(outs[1])
    out_vars = []
    for t0, t1 in zip(flat0, flat1):
        s0, s1 = list(t0._t.shape), list(t1._t.shape)
        shp = [a if a == b else -1 for a, b in zip(s0, s1)] if len(s0) == len(s1) else s0
        v = Variable(blk, shp, t0._t.dtype, stop_gradient=False)
        blk.vars[v.vid] = v
        out_vars.append(v)
    op = OpDesc(f'layer:{type(layer).__name__}', call, targs, tkw, in_vids,
                [v.vid for v in out_vars], tmpl)
    op.attrs['layer'] = layer
    op.attrs['params'] = list(layer.parameters())
    _record_amp(op)
    blk.ops.append(op)
    prog._bump()
    return _rebuild(tmpl, iter(out_vars))


_INSTALLED = [False]


def install_static_hooks():
    """Wrap every public paddle API function so calls on Variables are recorded."""
    if _INSTALLED[0]:
        return
    _INSTALLED[0] = True
    import types
    import paddle_ray_amd as P
    from ..tensor import creation, math, manipulation, linalg as tlinalg, random as trandom
    from ..nn import functional as NF
    from ..incubate.nn import functional as IF
    from .. import linalg as LA, metric as MET
    # paddle.fft records its own fft_c2c / fft_r2c / fft_c2r primitive ops
    modules = [creation, math, manipulation, tlinalg, trandom, NF, IF]
    mapping = {}
    for mod in modules:
        for name, obj in list(vars(mod).items()):
            if name.startswith('_') or not isinstance(obj, types.FunctionType):
                continue
            if obj.__module__ and not obj.__module__.startswith('paddle_ray_amd'):
                continue
            if name in ('seed', 'get_rng_state', 'set_rng_state', 'get_cuda_rng_state',
                        'set_cuda_rng_state', 'broadcast_shape', 'is_tensor', 'tolist',
                        'create_parameter', 'create_global_var'):
                continue
            w = static_op(f'{mod.__name__}:{name}', obj)
            mapping[id(obj)] = w
            setattr(mod, name, w)
    for ns in [P, P.tensor, LA, P.nn.functional]:
        for name, obj in list(vars(ns).items()):
            if isinstance(obj, types.FunctionType) and id(obj) in mapping:
                setattr(ns, name, mapping[id(obj)])
    for name, obj in list(vars(Tensor).items()):
        if isinstance(obj, types.FunctionType) and id(obj) in mapping:
            setattr(Tensor, name, mapping[id(obj)])

    # Variable operators record through the (wrapped) math functions
    def binop(fname, reverse=False):
        def op(self, other):
            f = getattr(math, fname)
            return f(other, self) if reverse else f(self, other)
        return op
    for dunder, fname in [('add', 'add'), ('sub', 'subtract'), ('mul', 'multiply'),
                          ('truediv', 'divide'), ('floordiv', 'floor_divide'),
                          ('mod', 'remainder'), ('pow', 'pow'), ('eq', 'equal'),
                          ('ne', 'not_equal'), ('lt', 'less_than'), ('le', 'less_equal'),
                          ('gt', 'greater_than'), ('ge', 'greater_equal'),
                          ('and', 'logical_and'), ('or', 'logical_or')]:
        setattr(Variable, f'__{dunder}__', binop(fname))
        if dunder in ('add', 'sub', 'mul', 'truediv', 'floordiv', 'mod', 'pow'):
            setattr(Variable, f'__r{dunder}__', binop(fname, True))
    Variable.__matmul__ = lambda self, o: tlinalg.matmul(self, o)
    Variable.__neg__ = lambda self: math.scale(self, -1.0)
    Variable.__getitem__ = lambda self, idx: static_op(
        'paddle_ray_amd.static.graph:_op_getitem', _op_getitem)(self, idx)
    Variable.__hash__ = lambda self: id(self)
