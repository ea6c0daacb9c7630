"""paddle.autograd (parity: python/paddle/autograd/{py_layer,backward_mode,saved_tensors_hooks}.py).

The eager tape is PyTorch-ROCm's autograd engine; ``PyLayer`` maps to a
``torch.autograd.Function`` whose ctx exposes the paddle PyLayerContext API.
"""
import torch

from ..framework.core import Tensor, _u, _w


def _wrap_tree(x):
    if isinstance(x, torch.Tensor):
        return Tensor(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_wrap_tree(e) for e in x)
    return x


def _unwrap_tree(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        return type(x)(_unwrap_tree(e) for e in x)
    return x


class PyLayerContext:
    def __init__(self, tctx):
        self._ctx = tctx
        self._saved = ()
        self.not_inplace_tensors = ()
        self.materialize_grads = True

    def save_for_backward(self, *tensors):
        self._ctx.save_for_backward(*[_u(t) for t in tensors])

    def saved_tensor(self):
        return tuple(Tensor(t) if t is not None else None for t in self._ctx.saved_tensors)

    def mark_not_inplace(self, *args):
        self.not_inplace_tensors = args

    def mark_non_differentiable(self, *args):
        self._ctx.mark_non_differentiable(*[_u(a) for a in args])

    def set_materialize_grads(self, value):
        self._ctx.set_materialize_grads(value)
        self.materialize_grads = value

    def __setattr__(self, k, v):
        if k in ('_ctx', '_saved', 'not_inplace_tensors', 'materialize_grads'):
            object.__setattr__(self, k, v)
        else:
            setattr(self._ctx, '_pl_' + k, v)

    def __getattr__(self, k):
        return getattr(self._ctx, '_pl_' + k)


class _PyLayerMeta(type):
    def __init__(cls, name, bases, attrs):
        super().__init__(name, bases, attrs)
        if name == 'PyLayer':
            return
        user_fwd, user_bwd = attrs.get('forward'), attrs.get('backward')

        class _Fn(torch.autograd.Function):
            @staticmethod
            def forward(tctx, *args):
                ctx = PyLayerContext(tctx)
                tctx._pl_ctx = ctx
                out = user_fwd(ctx, *_wrap_tree(args))
                return _unwrap_tree(out)

            @staticmethod
            def backward(tctx, *grads):
                ctx = tctx._pl_ctx
                res = user_bwd(ctx, *_wrap_tree(grads))
                if not isinstance(res, tuple):
                    res = (res,)
                res = _unwrap_tree(res)
                # pad with None for non-tensor forward args
                n = tctx._pl_nargs
                res = list(res)
                out = []
                it = iter(res)
                for is_t in tctx._pl_tensor_mask:
                    out.append(next(it, None) if is_t else None)
                return tuple(out[:n])

        cls._fn = _Fn


class PyLayer(metaclass=_PyLayerMeta):
    @classmethod
    def apply(cls, *args, **kwargs):
        targs = _unwrap_tree(args)
        mask = [isinstance(a, torch.Tensor) for a in targs]

        class _Bound(cls._fn):
            pass

        orig_forward = cls._fn.forward

        def fwd(tctx, *a):
            tctx._pl_nargs = len(a)
            tctx._pl_tensor_mask = mask
            return orig_forward(tctx, *a)
        _Bound.forward = staticmethod(fwd)
        out = _Bound.apply(*targs)
        return _wrap_tree(out)


def backward(tensors, grad_tensors=None, retain_graph=False):
    ts = [_u(t) for t in (tensors if isinstance(tensors, (list, tuple)) else [tensors])]
    gs = None
    if grad_tensors is not None:
        gs = [None if g is None else _u(g) for g in
              (grad_tensors if isinstance(grad_tensors, (list, tuple)) else [grad_tensors])]
    torch.autograd.backward(ts, gs, retain_graph=retain_graph)


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False,
         only_inputs=True, allow_unused=False, no_grad_vars=None):
    """paddle.grad (parity: python/paddle/fluid/dygraph/base.py:grad)."""
    single = not isinstance(inputs, (list, tuple))
    outs = [_u(o) for o in (outputs if isinstance(outputs, (list, tuple)) else [outputs])]
    ins = [_u(i) for i in ([inputs] if single else inputs)]
    gos = None
    if grad_outputs is not None:
        gos = [None if g is None else _u(g) for g in
               (grad_outputs if isinstance(grad_outputs, (list, tuple)) else [grad_outputs])]
    res = torch.autograd.grad(outs, ins, gos, retain_graph=retain_graph, create_graph=create_graph,
                              allow_unused=allow_unused)
    res = [None if r is None else Tensor(r) for r in res]
    return res


class saved_tensors_hooks:
    def __init__(self, pack_hook, unpack_hook):
        self._h = torch.autograd.graph.saved_tensors_hooks(
            lambda t: pack_hook(Tensor(t)), lambda x: _u(unpack_hook(x)))

    def __enter__(self):
        self._h.__enter__()
        return self

    def __exit__(self, *a):
        return self._h.__exit__(*a)


def jacobian(func, xs, batch_axis=None):
    x = _u(xs)
    return Tensor(torch.autograd.functional.jacobian(lambda t: _u(func(Tensor(t))), x))


def hessian(func, xs, batch_axis=None):
    x = _u(xs)
    return Tensor(torch.autograd.functional.hessian(lambda t: _u(func(Tensor(t))), x))
