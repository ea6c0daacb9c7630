"""paddle.incubate.passes (parity: python/paddle/incubate/passes/): graph passes.

``fuse_resnet_unit_pass`` (reference: incubate/passes/fuse_resnet_unit_pass.py, pattern
``relu(batch_norm(conv2d(x)))`` and ``relu(batch_norm(conv2d(x)) + batch_norm(conv2d(z)))``
rewritten into the cuDNN-v8 ``resnet_unit`` op) rewrites the same chains of a static
``Program`` into ONE op that runs the conv on the in-tree implicit-GEMM kernel and the
BatchNorm + residual add + ReLU as one statistics pass plus one fused apply pass
(``ops/csrc/bn.hip``) — the separate add / relu elementwise passes and their HBM round trips
disappear, and the ReLU backward reads 1 keep-bit per element instead of the output.

Also covered (beyond the reference's two patterns): ``relu(batch_norm(conv2d(x)) + z)`` with
any ``z`` (the unit's ``fuse_add``), and any NHWC/NCHW conv2d (not only 1x1). The rewrite is
applied to forward programs (before ``append_backward`` / ``minimize``, like the reference's
test applies it to a forward-only graph); ops that already carry grad ops are left alone.
"""
import inspect

from ...static import graph as G

_CONV = 'paddle_ray_amd.nn.functional:conv2d'
_BN = 'paddle_ray_amd.nn.functional:batch_norm'
_RELU = 'paddle_ray_amd.nn.functional:relu'
_ADDS = ('paddle_ray_amd.tensor.math:add',)
_FUSED = 'paddle_ray_amd.incubate.passes:conv_bn_add_act'


def conv_bn_add_act(x, conv_x, bn_x, z=None, conv_z=None, bn_z=None, act='relu'):
    """act(BN_x(conv_x(x)) + [BN_z(conv_z(z)) | z]) — the fused op the pass emits.
    ``conv_*`` / ``bn_*`` are the keyword arguments of the replaced conv2d / batch_norm ops
    (weights and running statistics included), so the op is exactly what it replaced."""
    from ...nn import functional as F

    def conv_bn(inp, ck, bk, res, a):
        c = F.conv2d(inp, **ck)
        training = bk.get('training', False) and not bk.get('use_global_stats')
        return F.fused_bn_add_act(c, res, bk['running_mean'], bk['running_var'], bk.get('weight'),
                                  bk.get('bias'), training, bk.get('momentum', 0.9),
                                  bk.get('epsilon', 1e-5), a,
                                  bk.get('data_format', 'NCHW'))
    short = z
    if conv_z is not None:
        short = conv_bn(z, conv_z, bn_z, None, None)
    return conv_bn(x, conv_x, bn_x, short, act)


G.register_static_op(_FUSED, conv_bn_add_act)


def _bind(op):
    """(first input, the op's other arguments by name) — positional args bound to names."""
    sig = inspect.signature(op.fn)
    b = sig.bind(*op.args, **op.kwargs)
    names = list(sig.parameters)
    kw = dict(b.arguments)
    for n, p in sig.parameters.items():  # flatten **kwargs
        if p.kind is inspect.Parameter.VAR_KEYWORD and n in kw:
            kw.update(kw.pop(n))
    first = kw.pop(names[0])
    kw.pop('name', None)
    return first, kw


def _refs(obj):
    if isinstance(obj, G._VarRef):
        yield obj.vid
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            yield from _refs(o)
    elif isinstance(obj, dict):
        for o in obj.values():
            yield from _refs(o)


def fuse_resnet_unit_pass(program=None):
    """Rewrite conv2d -> batch_norm (-> add) -> relu chains of ``program`` (default: the
    default main program) into fused ops. Returns the program; ``program._fused_resnet_units``
    counts the rewrites."""
    prog = program if program is not None else G.default_main_program()
    blk = prog.global_block()
    ops = blk.ops
    producer, users = {}, {}
    for op in ops:
        for v in op.out_vids:
            producer[v] = op
        for v in op.in_vids:
            users.setdefault(v, []).append(op)

    def only_user(vid, op):
        return users.get(vid, []) == [op]

    def single_out(op):
        return len(op.out_vids) == 1 and op.ctx_vid is None and op.role == 'forward'

    def conv_bn_of(vid, consumer):
        """(conv op, bn op, x ref, conv kw, bn kw) when vid = batch_norm(conv2d(x)) feeding
        only ``consumer``."""
        bn = producer.get(vid)
        if bn is None or bn.type != _BN or not single_out(bn) or not only_user(vid, consumer):
            return None
        xb, bkw = _bind(bn)
        if not isinstance(xb, G._VarRef) or bkw.get('data_format', 'NCHW') not in ('NHWC', 'NCHW'):
            return None
        conv = producer.get(xb.vid)
        if conv is None or conv.type != _CONV or not single_out(conv) or not only_user(xb.vid, bn):
            return None
        xc, ckw = _bind(conv)
        fmt = ckw.get('data_format', 'NCHW')
        if fmt != bkw.get('data_format', 'NCHW') or ckw.get('groups', 1) != 1:
            return None
        return conv, bn, xc, ckw, bkw

    removed, new_ops, fused = set(), {}, 0
    for relu in ops:
        if relu.type != _RELU or not single_out(relu) or len(relu.in_vids) != 1:
            continue
        rin = relu.in_vids[0]
        args = None
        main = conv_bn_of(rin, relu)
        if main is not None:
            conv, bn, xc, ckw, bkw = main
            chain = [conv, bn]
            args = dict(x=xc, conv_x=ckw, bn_x=bkw)
        else:
            add = producer.get(rin)
            if add is None or add.type not in _ADDS or not single_out(add) \
                    or not only_user(rin, relu) or len(add.args) < 2:
                continue
            a, b = add.args[0], add.args[1]
            ma = conv_bn_of(a.vid, add) if isinstance(a, G._VarRef) else None
            mb = conv_bn_of(b.vid, add) if isinstance(b, G._VarRef) else None
            if ma is None and mb is None:
                continue
            if ma is None:
                ma, mb, a, b = mb, ma, b, a
            conv, bn, xc, ckw, bkw = ma
            chain = [conv, bn, add]
            args = dict(x=xc, conv_x=ckw, bn_x=bkw)
            if mb is not None:  # shortcut branch: conv + BN of z
                chain += [mb[0], mb[1]]
                args.update(z=mb[2], conv_z=mb[3], bn_z=mb[4])
            else:  # plain residual
                args.update(z=b)
        in_vids = list(dict.fromkeys(_refs(args)))
        op = G.OpDesc(_FUSED, conv_bn_add_act, [], args, in_vids, list(relu.out_vids),
                      relu.out_template)
        op.attrs = dict(relu.attrs)
        op.attrs['params'] = [p for c in chain for p in c.attrs.get('params', [])]
        for c in chain:
            if 'amp' in c.attrs:
                op.attrs['amp'] = c.attrs['amp']
        for v in op.out_vids:
            blk.vars[v].__dict__['op'] = op
        removed.update(id(c) for c in chain)
        new_ops[id(relu)] = op
        fused += 1
    if fused:
        blk.ops = [new_ops.get(id(o), o) for o in ops if id(o) not in removed]
        prog._bump()
    prog._fused_resnet_units = getattr(prog, '_fused_resnet_units', 0) + fused
    return prog


__all__ = ['fuse_resnet_unit_pass']
