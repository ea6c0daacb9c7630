"""Op-fusion passes over ``paddle.static`` programs (parity: python/paddle/distributed/passes/
cpp_pass.py -- fuse_elewise_add_act :22, fused_feedforward :87, fuse_gemm_epilogue :100,
fuse_optimizer :113; the C++ graph passes they wrap, e.g. paddle/fluid/framework/ir/
fuse_gemm_epilogue_pass.cc, fused_feedforward_pass.cc).

The patterns are matched on this framework's own forward OpDescs and replaced by the ops of
static/fn_ops.py, i.e. by the in-tree HIP kernels with direct grad kernels:

* fuse_gemm_epilogue: ``linear -> gelu -> linear`` becomes ``fused_mlp_gelu`` (bias + GELU and
  its derivative inside the MFMA GEMM epilogues; the second bias stays a broadcast add);
  ``linear -> gelu`` becomes ``fused_linear`` + ``fused_bias_gelu`` (the bias rides the GELU
  kernel); every other 2-D-weight ``linear`` becomes ``fused_linear`` (fused bias / dW / db);
* fused_feedforward: the MLP rule above plus ``dropout(linear2) + residual -> layer_norm``
  becoming one ``fused_add_dropout_ln`` (bias + dropout + residual add + LayerNorm in one pass,
  the residual sum kept for the next block);
* fuse_elewise_add_act: ``x + bias -> gelu`` (bias a 1-D parameter over the last axis) becomes
  ``fused_bias_gelu``;
* fuse_optimizer: the optimize op already runs Adam(W) / Momentum as one multi-tensor kernel
  launch; the pass checks and marks it.

Intermediate variables a fusion removes can no longer be fetched. Programs that are already
minimized are stripped to their forward, fused, and re-minimized (static/graph.py
``rebuild_training``). Dropout inside ``fused_add_dropout_ln`` draws its mask from the kernel's
counter-based RNG, so a fused program matches the unfused one bit for bit only at p = 0."""
import inspect

from ...static import graph as G
from ...static import fn_ops as FO
from ...tensor import math as TM
from .pass_base import PassBase, PassType, register_pass

__all__ = []


def _name(op):
    mod, _, fn = op.type.rpartition(':')
    return fn if mod.startswith('paddle_ray_amd.') else None


def _bound(op):
    try:
        ba = inspect.signature(op.fn).bind(*op.args, **op.kwargs)
    except (TypeError, ValueError):
        return None
    ba.apply_defaults()
    return ba.arguments


def _is_param(a):
    return isinstance(a, G.Parameter)


class _Graph:
    """Consumers / producers of the forward ops of a block."""

    def __init__(self, blk):
        self.blk = blk
        self.consumers = {}
        for op in blk.ops:
            for v in op.in_vids:
                self.consumers.setdefault(v, []).append(op)

    def only_consumer(self, vid, op):
        c = self.consumers.get(vid, [])
        return len(c) == 1 and c[0] is op

    def single_consumer(self, vid):
        c = self.consumers.get(vid, [])
        return c[0] if len(c) == 1 else None


def _linear(op):
    """(x ref, W, b) of a plain 2-D-weight linear op, else None."""
    if _name(op) != 'linear' or len(op.out_vids) != 1:
        return None
    a = _bound(op)
    if a is None:
        return None
    x, w, b = a.get('x'), a.get('weight'), a.get('bias')
    if not isinstance(x, G._VarRef) or not _is_param(w) or G._u(w).dim() != 2:
        return None
    if b is not None and not (_is_param(b) and G._u(b).dim() == 1):
        return None
    return x, w, b


def _gelu(op):
    if _name(op) != 'gelu' or len(op.out_vids) != 1:
        return None
    a = _bound(op)
    if a is None or not isinstance(a.get('x'), G._VarRef):
        return None
    return a['x'], bool(a.get('approximate', False))


def _ref_vids(obj, out):
    if isinstance(obj, G._VarRef):
        if obj.vid not in out:
            out.append(obj.vid)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _ref_vids(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _ref_vids(o, out)
    return out


def _new_op(blk, op_type, fn, args, out_vids, template, like, params):
    in_vids = _ref_vids(list(args), [])
    op = G.OpDesc(op_type, fn, list(args), {}, in_vids, list(out_vids), template)
    op.attrs['params'] = [p for p in params if p is not None]
    for k in ('amp', 'device', 'recompute_id'):
        if k in like.attrs:
            op.attrs[k] = like.attrs[k]
    for v in out_vids:
        blk.vars[v].__dict__['op'] = op
    return op


def _replace(blk, old_ops, new_ops):
    """Put ``new_ops`` where the last of ``old_ops`` was and drop ``old_ops``."""
    pos = max(blk.ops.index(o) for o in old_ops)
    ids = {id(o) for o in old_ops}
    head = [o for o in blk.ops[:pos + 1] if id(o) not in ids]
    tail = blk.ops[pos + 1:]
    blk.ops[:] = head + list(new_ops) + tail


_F = {k: getattr(FO, k).__wrapped__ for k in ('fused_linear', 'fused_mlp_gelu', 'fused_bias_gelu',
                                              'fused_add_dropout_ln')}
_ADD_TYPE = next(t for t, f in G._OP_TABLE.items() if f is TM.add) if any(
    f is TM.add for f in G._OP_TABLE.values()) else 'paddle_ray_amd.tensor.math:add'


def _var(blk, vid):
    return blk.vars[vid]


def _tmp_like(blk, vid, name=None):
    v = blk.vars[vid]
    return G._new_var(blk, list(v._vshape), v.dtype, name)


def _fuse_mlp(blk, g, l1):
    """linear(x, W1, b1) -> gelu -> linear(., W2, b2) => fused_mlp_gelu (+ b2). Returns the new
    op producing the pre-bias output (or None), and b2."""
    p1 = _linear(l1)
    if p1 is None or p1[2] is None:
        return None
    ge = g.single_consumer(l1.out_vids[0])
    if ge is None or _gelu(ge) is None or _gelu(ge)[0].vid != l1.out_vids[0]:
        return None
    l2 = g.single_consumer(ge.out_vids[0])
    p2 = _linear(l2) if l2 is not None else None
    if p2 is None or p2[0].vid != ge.out_vids[0]:
        return None
    x, w1, b1 = p1
    _, w2, b2 = p2
    return ge, l2, x, w1, b1, w2, b2, _gelu(ge)[1]


def fuse_gemm_epilogue(prog, mlp=True, linear_gelu=True, plain=True):
    blk = prog.global_block()
    n = 0
    if mlp:
        for l1 in list(blk.ops):
            if not any(o is l1 for o in blk.ops):
                continue
            m = _fuse_mlp(blk, _Graph(blk), l1)
            if m is None:
                continue
            ge, l2, x, w1, b1, w2, b2, approx = m
            out = l2.out_vids[0]
            if b2 is None:
                fused = _new_op(blk, 'fused_mlp_gelu', _F['fused_mlp_gelu'], [x, w1, b1, w2, approx],
                                [out], 'T', l1, [w1, b1, w2])
                _replace(blk, [l1, ge, l2], [fused])
            else:
                h = _tmp_like(blk, out)
                fused = _new_op(blk, 'fused_mlp_gelu', _F['fused_mlp_gelu'], [x, w1, b1, w2, approx],
                                [h.vid], 'T', l1, [w1, b1, w2])
                add = _new_op(blk, _ADD_TYPE, TM.add, [G._VarRef(h.vid), b2], [out], 'T', l2, [b2])
                _replace(blk, [l1, ge, l2], [fused, add])
            n += 1
    if linear_gelu:
        for lin in list(blk.ops):
            if not any(o is lin for o in blk.ops):
                continue
            p = _linear(lin)
            if p is None or p[2] is None:
                continue
            g = _Graph(blk)
            ge = g.single_consumer(lin.out_vids[0])
            if ge is None or _gelu(ge) is None:
                continue
            x, w, b = p
            t = _tmp_like(blk, lin.out_vids[0])
            f1 = _new_op(blk, 'fused_linear', _F['fused_linear'], [x, w, None], [t.vid], 'T', lin, [w])
            f2 = _new_op(blk, 'fused_bias_gelu', _F['fused_bias_gelu'], [G._VarRef(t.vid), b, _gelu(ge)[1]],
                         [ge.out_vids[0]], 'T', ge, [b])
            _replace(blk, [lin, ge], [f1, f2])
            n += 1
    if plain:
        for lin in list(blk.ops):
            p = _linear(lin)
            if p is None:
                continue
            x, w, b = p
            f = _new_op(blk, 'fused_linear', _F['fused_linear'], [x, w, b], [lin.out_vids[0]], 'T',
                        lin, [w, b])
            _replace(blk, [lin], [f])
            n += 1
    return n


def _dropout(op):
    if _name(op) != 'dropout' or len(op.out_vids) != 1:
        return None
    a = _bound(op)
    if a is None or not isinstance(a.get('x'), G._VarRef) or a.get('axis') is not None or \
            a.get('mode', 'upscale_in_train') != 'upscale_in_train':
        return None
    p = float(a.get('p', 0.5)) if a.get('training', True) else 0.0
    return a['x'], p


def _add2(op):
    if _name(op) != 'add' or len(op.out_vids) != 1:
        return None
    a = list(op.args)
    if len(a) != 2 or op.kwargs or not all(isinstance(t, G._VarRef) for t in a):
        return None
    return a


def _layer_norm(op):
    if _name(op) != 'layer_norm' or len(op.out_vids) != 1:
        return None
    a = _bound(op)
    if a is None or not isinstance(a.get('x'), G._VarRef):
        return None
    shp = a.get('normalized_shape')
    shp = [shp] if isinstance(shp, int) else list(shp or [])
    w, b = a.get('weight'), a.get('bias')
    if len(shp) != 1 or not _is_param(w) or not _is_param(b):
        return None
    return a['x'], w, b, float(a.get('epsilon', 1e-5))


def _producer(blk, vid):
    v = blk.vars.get(vid)
    op = v.__dict__.get('op') if v is not None else None
    return op if op is not None and any(o is op for o in blk.ops) else None


def fuse_feedforward(prog):
    """MLP fusion + ``linear2 -> dropout -> (+ residual) -> layer_norm`` => fused_add_dropout_ln."""
    blk = prog.global_block()
    n = 0
    for dp in list(blk.ops):
        if not any(o is dp for o in blk.ops):
            continue
        d = _dropout(dp)
        if d is None:
            continue
        g = _Graph(blk)
        lin = _producer(blk, d[0].vid)
        p2 = _linear(lin) if lin is not None else None
        if p2 is None or not g.only_consumer(d[0].vid, dp):
            continue
        add = g.single_consumer(dp.out_vids[0])
        a2 = _add2(add) if add is not None else None
        if a2 is None:
            continue
        res = a2[0] if a2[1].vid == dp.out_vids[0] else a2[1]
        if res.vid == dp.out_vids[0]:
            continue
        lns = [o for o in g.consumers.get(add.out_vids[0], []) if _layer_norm(o) is not None and
               _layer_norm(o)[0].vid == add.out_vids[0]]
        if len(lns) != 1:
            continue
        ln = lns[0]
        _, lw, lb, eps = _layer_norm(ln)
        # the FFN up-projection + GELU in front of this projection folds in as one MLP op
        ml = None
        ge = _producer(blk, p2[0].vid)
        if ge is not None and _gelu(ge) is not None:
            up = _producer(blk, _gelu(ge)[0].vid)
            m = _fuse_mlp(blk, g, up) if up is not None else None
            if m is not None and m[1] is lin:
                ml = (up, m)
        x2, w2, b2 = p2
        h = _tmp_like(blk, lin.out_vids[0])
        if ml is not None:
            up, (ge, _, x, w1, b1, _, _, approx) = ml
            first = _new_op(blk, 'fused_mlp_gelu', _F['fused_mlp_gelu'], [x, w1, b1, w2, approx],
                            [h.vid], 'T', up, [w1, b1, w2])
            olds = [up, ge, lin]
        else:
            first = _new_op(blk, 'fused_linear', _F['fused_linear'], [x2, w2, None], [h.vid], 'T', lin, [w2])
            olds = [lin]
        adl = _new_op(blk, 'fused_add_dropout_ln', _F['fused_add_dropout_ln'],
                      [res, G._VarRef(h.vid), b2, lw, lb, d[1], eps], [add.out_vids[0], ln.out_vids[0]],
                      ('tuple', ['T', 'T']), ln, [b2, lw, lb])
        _replace(blk, olds + [dp, add, ln], [first, adl])
        n += 1
    # the remaining MLPs (no dropout / LayerNorm tail)
    n += fuse_gemm_epilogue(prog, mlp=True, linear_gelu=False, plain=False)
    return n


def fuse_elewise_add_act(prog):
    blk = prog.global_block()
    n = 0
    for add in list(blk.ops):
        if not any(o is add for o in blk.ops) or _name(add) != 'add' or len(add.args) != 2 or add.kwargs:
            continue
        a, b = add.args
        if _is_param(a) and isinstance(b, G._VarRef):
            a, b = b, a
        if not (isinstance(a, G._VarRef) and _is_param(b) and G._u(b).dim() == 1):
            continue
        xv = _var(blk, a.vid)
        if not xv._vshape or xv._vshape[-1] != G._u(b).shape[0]:
            continue
        g = _Graph(blk)
        ge = g.single_consumer(add.out_vids[0])
        if ge is None or _gelu(ge) is None:
            continue
        f = _new_op(blk, 'fused_bias_gelu', _F['fused_bias_gelu'], [a, b, _gelu(ge)[1]],
                    [ge.out_vids[0]], 'T', ge, [b])
        _replace(blk, [add, ge], [f])
        n += 1
    return n


class _FusionPass(PassBase):
    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        meta = main_program.__dict__.get('_train_meta')
        rebuild = meta['rebuild'] if meta is not None else None
        if meta is not None:
            G.strip_training(main_program)
        n = self._fuse(main_program)
        context.set_attr(f'{self.name}_count', (context.get_attr(f'{self.name}_count') or 0) + n)
        main_program._bump()
        if rebuild is not None:
            rebuild()

    def _fuse(self, prog):
        raise NotImplementedError


@register_pass('fuse_gemm_epilogue')
class FuseGemmEpiloguePass(_FusionPass):
    def _fuse(self, prog):
        return fuse_gemm_epilogue(prog)


@register_pass('fused_feedforward')
class FusedFeedforwardPass(_FusionPass):
    def _fuse(self, prog):
        return fuse_feedforward(prog)


@register_pass('fuse_elewise_add_act')
class FuseElewiseAddActPass(_FusionPass):
    def _fuse(self, prog):
        return fuse_elewise_add_act(prog)


@register_pass('fuse_optimizer')
class FuseOptimizerPass(_FusionPass):
    """The reference fuses per-parameter adam / momentum / sgd ops into one. Here the optimize
    op already hands every parameter to ONE multi-tensor HIP launch for Adam / AdamW / Momentum
    (optimizer.py ``MultiTensorAdamW`` / ``momentum_mt``); the pass checks that and marks the
    op (``attrs['fused_optimizer']``). Other optimizers (SGD, Lamb, ...) run torch foreach
    updates; they are listed in the context attribute ``fuse_optimizer_unfused``."""

    def _apply_single_impl(self, main_program, startup_program, context):
        from ... import optimizer as O
        fused, unfused = 0, []
        for op in main_program.global_block().ops:
            if op.role != 'optimize':
                continue
            opt = next((a for a in op.args if hasattr(a, '_param_groups')), None)
            opt = G._inner_opt(opt) if opt is not None else None
            if opt is None:
                continue
            if isinstance(opt, (O.Adam, O.Momentum)) and not isinstance(opt, O.Lamb):
                op.attrs['fused_optimizer'] = True
                fused += 1
            else:
                unfused.append(type(opt).__name__)
        context.set_attr('fuse_optimizer_count', fused)
        context.set_attr('fuse_optimizer_unfused', unfused)
