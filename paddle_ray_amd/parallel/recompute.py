"""Activation recompute (parity: python/paddle/distributed/fleet/recompute/recompute.py).

Forward runs under no_grad keeping only the inputs; backward re-runs the
function with the SAME RNG state (CPU + every HIP device, and the TP RNG
tracker) so dropout masks match, then back-propagates through it.
"""
import torch

from ..framework.core import Tensor, _u
from .tensor_parallel import get_rng_state_tracker


_DEPTH = [0]
_DEFERRED = []


def queue_outer_callback(cb):
    """Queue ``cb`` to run when the OUTERMOST backward finishes. Inside a recompute backward
    (a nested, reentrant ``torch.autograd.backward``) the engine's callback queue belongs to
    the nested graph task, which ends after one block — the gradient reducers' end-of-backward
    hooks must wait for the outer one."""
    if _DEPTH[0] > 0:
        _DEFERRED.append(cb)
    else:
        torch.autograd.Variable._execution_engine.queue_callback(cb)


def _wrap(x):
    if isinstance(x, torch.Tensor):
        return Tensor(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_wrap(e) for e in x)
    return x


def _unwrap(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        return type(x)(_unwrap(e) for e in x)
    return x


class _RecomputeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fn, preserve, n_in, *args):
        ctx.fn, ctx.preserve = fn, preserve
        if preserve:
            ctx.cpu_state = torch.get_rng_state()
            ctx.dev_state = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
            ctx.tracker = get_rng_state_tracker().get_states_tracker()
        tensors, ctx.layout = [], []
        for a in args:
            if isinstance(a, torch.Tensor):
                tensors.append(a)
                ctx.layout.append(None)
            else:
                ctx.layout.append(a)
        ctx.save_for_backward(*tensors)
        with torch.no_grad():
            out = fn(*_wrap(args))
        out = _unwrap(out)
        ctx.tuple_out = isinstance(out, tuple)
        return out

    @staticmethod
    def backward(ctx, *grads):
        tens = list(ctx.saved_tensors)
        it = iter(tens)
        args = []
        for l in ctx.layout:
            if l is None:
                t = next(it)
                d = t.detach()
                d.requires_grad_(t.requires_grad)
                args.append(d)
            else:
                args.append(l)
        if ctx.preserve:
            cpu = torch.get_rng_state()
            dev = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
            trk = get_rng_state_tracker().get_states_tracker()
            torch.set_rng_state(ctx.cpu_state)
            if ctx.dev_state is not None:
                torch.cuda.set_rng_state(ctx.dev_state)
            get_rng_state_tracker().set_states_tracker(ctx.tracker)
        try:
            with torch.enable_grad():
                out = _unwrap(ctx.fn(*_wrap(tuple(args))))
        finally:
            if ctx.preserve:
                torch.set_rng_state(cpu)
                if dev is not None:
                    torch.cuda.set_rng_state(dev)
                get_rng_state_tracker().set_states_tracker(trk)
        outs = out if isinstance(out, tuple) else (out,)
        pairs = [(o, g) for o, g in zip(outs, grads)
                 if isinstance(o, torch.Tensor) and o.requires_grad and g is not None]
        if pairs:
            _DEPTH[0] += 1
            try:
                torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
            finally:
                _DEPTH[0] -= 1
            if _DEPTH[0] == 0 and _DEFERRED:
                cbs = list(_DEFERRED)
                _DEFERRED.clear()
                for cb in cbs:  # now on the outer graph task
                    torch.autograd.Variable._execution_engine.queue_callback(cb)
        in_grads = tuple(a.grad if isinstance(a, torch.Tensor) else None for a in args)
        return (None, None, None) + in_grads


def recompute(function, *args, **kwargs):
    preserve = kwargs.pop('preserve_rng_state', True)
    kwargs.pop('use_reentrant', None)
    if kwargs:
        fn0 = function
        function = lambda *a: fn0(*a, **kwargs)  # noqa: E731
    targs = _unwrap(args)
    if not torch.is_grad_enabled() or not any(isinstance(a, torch.Tensor) and a.requires_grad
                                              for a in targs):
        # parameters inside still need grads: use the reentrant path regardless
        pass
    out = _RecomputeFn.apply(function, preserve, len(targs), *targs)
    return _wrap(out)


def recompute_sequential(ctx, functions, *args, **kwargs):
    segments = ctx.get('segments', 1)
    layers = list(functions.children()) if hasattr(functions, 'children') else list(functions)
    per = max(1, len(layers) // segments)

    def run(lo, hi):
        def f(*xs):
            x = xs[0] if len(xs) == 1 else xs
            for l in layers[lo:hi]:
                x = l(x)
            return x
        return f
    x = args
    for lo in range(0, len(layers), per):
        x = recompute(run(lo, min(lo + per, len(layers))), *(x if isinstance(x, tuple) else (x,)))
    return x


def recompute_hybrid(ctx, function, *args, **kwargs):
    return recompute(function, *args, **kwargs)
