"""paddle.incubate.autograd (parity: python/paddle/incubate/autograd/__init__.py): functional
vjp / jvp, lazy Jacobian / Hessian, forward_grad / grad, and the prim switches.

Prim mode in the reference lowers static programs to primitive ops so that the transpose /
linearize rules produce higher-order derivatives. Here higher-order derivatives come from the
autograd engine directly (dygraph) and from grad ops of grad ops (static ``gradients``), so the
switch only records the user's choice (``prim_enabled``); ``forward_grad`` / ``grad`` work with
it on or off."""
import torch

from ...framework.core import Tensor, _u
from .functional import Hessian, Jacobian, jvp, vjp  # noqa: F401

__all__ = ['vjp', 'jvp', 'Jacobian', 'Hessian', 'enable_prim', 'disable_prim', 'forward_grad', 'grad']

_PRIM = [False]


def enable_prim():
    _PRIM[0] = True


def disable_prim():
    _PRIM[0] = False


def prim_enabled():
    return _PRIM[0]


def _list(x):
    return (list(x), False) if isinstance(x, (list, tuple)) else ([x], True)


def forward_grad(outputs, inputs, grad_inputs=None):
    """Forward-mode derivative d(outputs)/d(inputs) · grad_inputs (primapi.py:25) of outputs
    already computed from ``inputs`` (grad_inputs default: ones)."""
    from ...static import _static_mode_enabled
    if _static_mode_enabled():
        raise NotImplementedError("incubate.autograd.forward_grad runs in dygraph mode here; "
                                  "build the static program's derivative with static.gradients")
    ys, ysingle = _list(outputs)
    xs, _ = _list(inputs)
    yt, xt = [_u(y) for y in ys], [_u(x) for x in xs]
    if grad_inputs is None:
        tang = [torch.ones_like(x) for x in xt]
    else:
        gi, _ = _list(grad_inputs)
        tang = [_u(g).to(x.dtype) for g, x in zip(gi, xt)]
    ws = [torch.zeros_like(y, requires_grad=True) for y in yt]
    g = torch.autograd.grad(yt, xt, ws, create_graph=True, allow_unused=True)
    g = [torch.zeros_like(x) if gi is None else gi for gi, x in zip(g, xt)]
    if not any(gi.requires_grad for gi in g):
        out = [torch.zeros_like(y) for y in yt]
    else:
        pairs = [(gi, t) for gi, t in zip(g, tang) if gi.requires_grad]
        out = torch.autograd.grad([p for p, _ in pairs], ws, [t for _, t in pairs], allow_unused=True)
        out = [torch.zeros_like(y) if o is None else o for o, y in zip(out, yt)]
    out = [Tensor(o) for o in out]
    return out[0] if ysingle else out


def grad(outputs, inputs, grad_outputs=None):
    """Reverse-mode gradients of ``outputs`` w.r.t. ``inputs`` (primapi.py:108); in static mode
    the program gains the grad ops (static.gradients)."""
    from ...static import _static_mode_enabled
    if _static_mode_enabled():
        from ...static import gradients
        return gradients(outputs, inputs, grad_outputs)
    ys, _ = _list(outputs)
    xs, xsingle = _list(inputs)
    yt, xt = [_u(y) for y in ys], [_u(x) for x in xs]
    gos = [torch.ones_like(y) for y in yt] if grad_outputs is None else \
        [_u(g).to(y.dtype) for g, y in zip(_list(grad_outputs)[0], yt)]
    gs = torch.autograd.grad(yt, xt, gos, allow_unused=True, create_graph=torch.is_grad_enabled())
    out = [Tensor(torch.zeros_like(x) if g is None else g) for g, x in zip(gs, xt)]
    return out[0] if xsingle else out
