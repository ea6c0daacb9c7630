"""Static-graph control flow with run-time semantics: ``while_loop``, ``cond`` and
``StaticRNN`` build SUB-BLOCKS and execute them when the program runs.

Parity: python/paddle/static/nn/control_flow.py (while_loop -> ``while`` op over a sub-block,
cond -> two ``conditional_block`` ops + select_input, StaticRNN -> ``recurrent`` op) executed
by paddle/fluid/operators/controlflow/while_op.cc / conditional_block_op.cc /
recurrent_op.cc.

Each construct traces its Python callables ONCE into a sub-Program (placeholders stand for
the loop / step variables), then records a single op in the enclosing program. At run time
that op interprets its sub-block: the trip count and the branch taken depend on the fed
values, not on build-time values. Outer Variables the sub-block reads are passed to the op
as inputs (the planner keeps them alive), parameters it uses are registered with the
enclosing program, and autograd runs straight through the executed iterations — so
``append_backward`` yields the ``while_grad`` / ``conditional_block_grad`` equivalents via
the op's recorded VJP.
"""
import contextlib

import torch

from ..framework.core import Tensor, Parameter, _u
from . import graph as G


def _in_static(*objs):
    """Building a static program: loop vars may be Variables or constants created in it."""
    return bool(G._STATIC[0])


def _flat(out):
    if isinstance(out, (list, tuple)):
        r = []
        for o in out:
            r += _flat(o)
        return r
    return [out]


class _SubBlock:
    """A traced sub-program: placeholders -> outputs, plus captured outer Variables. It is
    an argument of the control-flow op that runs it and serializes as a nested op list
    (graph._encode ``__block__``; the ProgramDesc sub-block of the reference)."""
    _pra_block = True

    def __init__(self, outer_prog):
        self.prog = G.Program()
        self.outer = outer_prog
        self.placeholders = []

    def placeholder(self, like, shape=None):
        shp = list(like.shape) if shape is None else list(shape)
        v = G.Variable(self.prog.global_block(), shp, like.dtype, stop_gradient=False)
        self.prog.global_block().vars[v.vid] = v
        self.placeholders.append(v)
        return v

    @contextlib.contextmanager
    def tracing(self):
        with G.program_guard(self.prog):
            yield

    def finish(self, outputs):
        """Resolve captured outer Variables and parameters after tracing."""
        blk = self.prog.global_block()
        produced = {v.vid for v in self.placeholders}
        for op in blk.ops:
            produced.update(op.all_outputs())
        captured = {}
        # anything read but not produced here comes from an enclosing block (possibly
        # several levels out for nested control flow: the enclosing sub-blocks capture it too)
        for op in blk.ops:
            for vid in op.in_vids:
                if vid not in produced and vid in G._ALL_VARS:
                    captured[vid] = G._ALL_VARS[vid]
        for o in _flat(outputs):  # an output that IS an outer variable (identity body)
            if isinstance(o, G.Variable) and o.vid not in produced:
                captured[o.vid] = o
        self.captured = list(captured.values())
        self.params = list(self.prog._params.values())
        for p in self.params:
            self.outer._register_param(p)
        self.outputs = outputs
        return self

    @property
    def ph_vids(self):
        return [v.vid for v in self.placeholders]

    @property
    def cap_vids(self):
        return [v.vid for v in self.captured]

    def block_ops(self):
        return self.prog.global_block().ops

    def run(self, feed_vals, captured_vals, out_obj=None):
        """Execute the sub-block eagerly; returns the values of ``out_obj`` (default: the
        traced outputs)."""
        env = {v.vid: t for v, t in zip(self.placeholders, feed_vals)}
        env.update({v.vid: t for v, t in zip(self.captured, captured_vals)})
        return G.run_block_ops(self.block_ops(), env, self.outputs if out_obj is None else out_obj)


def _resolve(obj, env):
    if isinstance(obj, G.Variable):
        return env[obj.vid]
    if isinstance(obj, (list, tuple)):
        return type(obj)(_resolve(o, env) for o in obj)
    return obj


def _spec(v):
    return (list(v.shape), v.dtype)


def _tmpl_of(obj):
    _, tmpl = G._flatten_out(obj if not isinstance(obj, G.Variable) else obj)
    return tmpl


# -- while_loop --------------------------------------------------------------------------------
def while_loop(cond, body, loop_vars, is_test=False, name=None):
    """Repeat ``loop_vars = body(*loop_vars)`` while ``cond(*loop_vars)`` is true."""
    loop_vars = list(loop_vars)
    if not _in_static(loop_vars):
        vs = loop_vars
        while bool(_u(cond(*vs)).reshape(-1)[0]):
            out = body(*vs)
            vs = list(out) if isinstance(out, (list, tuple)) else [out]
        return vs
    prog = G.default_main_program()
    cb = _SubBlock(prog)
    bb = _SubBlock(prog)
    with cb.tracing():
        cps = [cb.placeholder(v) for v in loop_vars]
        c = cond(*cps)
    with bb.tracing():
        bps = [bb.placeholder(v) for v in loop_vars]
        out = body(*bps)
        out = list(out) if isinstance(out, (list, tuple)) else [out]
    if len(out) != len(loop_vars):
        raise ValueError(f"while_loop body returned {len(out)} values for {len(loop_vars)} "
                         f"loop vars")
    cb.finish(c)
    bb.finish(out)
    nl, ncc = len(loop_vars), len(cb.captured)
    args = [cb, bb, nl, ncc] + loop_vars + cb.captured + bb.captured + [cb.params + bb.params]
    specs = [_spec(v) for v in loop_vars]
    tmpl = ('tuple', ['T'] * nl)
    outs = G.record_op('while', while_op, args, {}, out_specs=(tmpl, specs))
    return list(outs)


def while_op(cb, bb, nl, ncc, *vals):
    """The ``while`` op (parity: controlflow/while_op.cc): re-run the body sub-block while the
    condition sub-block yields true. ``vals`` = loop vars, captured inputs of the condition,
    of the body, then the parameter list (an input for the planner only)."""
    vals = vals[:-1]
    vs = list(vals[:nl])
    c_cap = vals[nl:nl + ncc]
    b_cap = vals[nl + ncc:]
    while bool(_u(cb.run(vs, c_cap)).reshape(-1)[0]):
        vs = list(bb.run(vs, b_cap))
    return tuple(vs)


def conditional_block_op(pred, tb, fb, nt, *caps):
    """The ``conditional_block`` op (parity: controlflow/conditional_block_op.cc + select_input):
    run the sub-block of the branch ``pred`` selects. ``caps`` = captured inputs of the true
    block, of the false block, then the parameter list."""
    caps = caps[:-1]
    take = bool(_u(pred).reshape(-1)[0])
    out = tb.run([], caps[:nt]) if take else fb.run([], caps[nt:])
    flat = _flat(out)
    # an output that is a plain outer value/constant keeps its own tensor
    return tuple(o if isinstance(o, Tensor) else Tensor(torch.as_tensor(o)) for o in flat)


for _f in (while_op, conditional_block_op):
    G.register_static_op(f'{_f.__module__}:{_f.__qualname__}', _f)


# -- cond --------------------------------------------------------------------------------------
def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    """Run ``true_fn()`` if ``pred`` else ``false_fn()`` — only the taken branch executes."""
    if not (G._STATIC[0] and isinstance(pred, G.Variable)):
        p = bool(_u(pred).reshape(-1)[0]) if isinstance(pred, Tensor) else bool(pred)
        fn = true_fn if p else false_fn
        return fn() if fn is not None else None
    prog = G.default_main_program()
    tb, fb = _SubBlock(prog), _SubBlock(prog)
    with tb.tracing():
        t_out = true_fn() if true_fn is not None else None
    with fb.tracing():
        f_out = false_fn() if false_fn is not None else None
    if t_out is None or f_out is None:
        if t_out is None and f_out is None:
            return None
        raise ValueError("cond: both branches must return values (or both None)")
    tf, ff = _flat(t_out), _flat(f_out)
    if len(tf) != len(ff):
        raise ValueError(f"cond: true_fn returns {len(tf)} values, false_fn {len(ff)}")
    for a, b in zip(tf, ff):
        if list(a.shape) != list(b.shape) and -1 not in list(a.shape) + list(b.shape):
            raise ValueError(f"cond: branch outputs differ in shape {a.shape} vs {b.shape}")
    tb.finish(t_out)
    fb.finish(f_out)
    nt = len(tb.captured)
    args = [pred, tb, fb, nt] + tb.captured + fb.captured + [tb.params + fb.params]
    specs = [_spec(v) for v in tf]
    outs = G.record_op('conditional_block', conditional_block_op, args, {},
                       out_specs=(('tuple', ['T'] * len(tf)), specs))
    it = iter(outs)
    return G._rebuild(G._flatten_out(t_out)[1], it) if isinstance(t_out, (list, tuple)) \
        else next(it)


# -- StaticRNN ---------------------------------------------------------------------------------
class StaticRNN:
    """Time-major recurrent sub-block (parity: fluid StaticRNN):

        rnn = StaticRNN()
        with rnn.step():
            x_t = rnn.step_input(x)                   # x: [T, B, ...]
            h = rnn.memory(init=h0)                   # or memory(shape=, batch_ref=)
            h_new = ...
            rnn.update_memory(h, h_new)
            rnn.step_output(h_new)
        out = rnn()                                   # [T, B, ...]
    """

    def __init__(self, name=None):
        self._blk = None
        self._inputs, self._mems, self._updates, self._outputs = [], [], {}, []
        self._built = None

    @contextlib.contextmanager
    def step(self):
        self._blk = _SubBlock(G.default_main_program())
        with self._blk.tracing():
            yield
        self._finish()

    def step_input(self, x):
        v = self._blk.placeholder(x, shape=list(x.shape)[1:])
        self._inputs.append((x, v))
        return v

    def memory(self, init=None, shape=None, batch_ref=None, init_value=0.0, init_batch_dim_idx=0,
               ref_batch_dim_idx=1):
        if init is not None:
            v = self._blk.placeholder(init)
            self._mems.append((v, ('init', init)))
            return v
        if shape is None or batch_ref is None:
            raise ValueError("StaticRNN.memory needs init, or shape and batch_ref")
        shp = list(shape)
        v = G.Variable(self._blk.prog.global_block(), shp, batch_ref.dtype, stop_gradient=False)
        self._blk.prog.global_block().vars[v.vid] = v
        self._blk.placeholders.append(v)
        # batch size comes from the step input at run time
        self._mems.append((v, ('fill', shp, float(init_value), batch_ref, ref_batch_dim_idx,
                               init_batch_dim_idx)))
        return v

    def update_memory(self, mem, var):
        self._updates[mem.vid] = var

    def step_output(self, o):
        self._outputs.append(o)

    def output(self, *outputs):
        for o in outputs:
            self.step_output(o)

    def _finish(self):
        missing = [m for m, _ in self._mems if m.vid not in self._updates]
        if missing:
            raise ValueError("StaticRNN: every memory needs update_memory()")
        blk = self._blk
        tracked = self._outputs + [self._updates[m.vid] for m, _ in self._mems]
        blk.finish(tracked)
        xs = [x for x, _ in self._inputs]
        inits = [spec[1] for _, spec in self._mems if spec[0] == 'init']
        n_in, n_init, n_out, n_mem = len(xs), len(inits), len(self._outputs), len(self._mems)
        mem_specs = [spec for _, spec in self._mems]

        def run_rnn(*vals):
            seqs = [_u(v) for v in vals[:n_in]]
            init_vals = list(vals[n_in:n_in + n_init])
            caps = vals[n_in + n_init:]
            T = seqs[0].shape[0]
            mems, it = [], iter(init_vals)
            for spec in mem_specs:
                if spec[0] == 'init':
                    mems.append(next(it))
                else:
                    _, shp, val, ref, ref_dim, init_dim = spec
                    b = seqs[[id(x) for x in xs].index(id(ref))].shape[ref_dim] \
                        if any(x is ref for x in xs) else seqs[0].shape[1]
                    full = [b if (i == init_dim and s < 0) else s for i, s in enumerate(shp)]
                    mems.append(Tensor(torch.full(full, val, dtype=seqs[0].dtype,
                                                  device=seqs[0].device)))
            outs = [[] for _ in range(n_out)]
            for t in range(T):
                feed = [Tensor(s[t]) for s in seqs] + mems
                res = blk.run(feed, caps)
                for k in range(n_out):
                    outs[k].append(_u(res[k]))
                mems = list(res[n_out:n_out + n_mem])
            return tuple(Tensor(torch.stack(o, 0)) for o in outs)
        args = xs + inits + blk.captured + [blk.params]
        T0 = xs[0].shape[0] if xs else -1
        specs = [([T0] + list(o.shape), o.dtype) for o in self._outputs]
        outs = G.record_op('recurrent', lambda *a: run_rnn(*a[:-1]), args, {},
                           out_specs=(('tuple', ['T'] * n_out), specs))
        self._built = list(outs)

    def __call__(self, *args, **kwargs):
        if self._built is None:
            raise ValueError("StaticRNN: call after the `with rnn.step():` block")
        return self._built[0] if len(self._built) == 1 else self._built
