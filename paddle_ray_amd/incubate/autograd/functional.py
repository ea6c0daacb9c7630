"""Functional higher-order autodiff (parity: python/paddle/incubate/autograd/functional.py --
vjp :22, jvp :80, the lazy Jacobian :171 / Hessian :260 with ``is_batched``; primapi.py:25,108
forward_grad / grad).

Everything runs on the autograd engine of the eager tensors (reverse mode; forward-mode
products by the double-backward construction: for u with dy = J u, differentiate
<grad(y, x, w), u> with respect to the dummy cotangent w). Jacobian / Hessian objects are LAZY:
indexing evaluates only the rows it needs (one reverse pass per row of the lazy axis) and caches
them; ``J[:]`` materialises the whole matrix."""
import torch

from ...framework.core import Tensor, _u

__all__ = ['vjp', 'jvp', 'Jacobian', 'Hessian']


def _as_list(xs):
    if isinstance(xs, (list, tuple)):
        return list(xs), False
    return [xs], True


def _leaf(x, keep_graph=False):
    t = _u(x)
    if keep_graph:
        if not t.requires_grad:
            t = t.detach().requires_grad_(True)
        return t
    return t.detach().clone().requires_grad_(True)


def _grads(ys, xs, cot, create_graph=False, retain_graph=True):
    pairs = [(y, c) for y, c in zip(ys, cot) if y.requires_grad]
    if not pairs:
        return [torch.zeros_like(x) for x in xs]
    gs = torch.autograd.grad([y for y, _ in pairs], xs, [c for _, c in pairs], create_graph=create_graph,
                             retain_graph=retain_graph, allow_unused=True)
    return [torch.zeros_like(x) if g is None else g for g, x in zip(gs, xs)]


def _check_v(v, refs, what):
    vs, _ = _as_list(v)
    if len(vs) != len(refs):
        raise ValueError(f"{what}: expected {len(refs)} tensors in v, got {len(vs)}")
    out = []
    for a, r in zip(vs, refs):
        a = _u(a)
        if tuple(a.shape) != tuple(r.shape):
            raise ValueError(f"{what}: v shape {tuple(a.shape)} does not match {tuple(r.shape)}")
        out.append(a.to(r.dtype))
    return out


def vjp(func, xs, v=None):
    """(func(xs), vᵀ·J): the vector-Jacobian product; v defaults to ones like the outputs."""
    xl, single = _as_list(xs)
    leaves = [_leaf(x) for x in xl]
    ys = func(*[Tensor(t) for t in leaves])
    yl, ysingle = _as_list(ys)
    yt = [_u(y) for y in yl]
    cot = [torch.ones_like(y) for y in yt] if v is None else _check_v(v, yt, 'vjp')
    gs = [Tensor(g) for g in _grads(yt, leaves, cot, retain_graph=False)]
    return ys, (gs[0] if single else gs)


def jvp(func, xs, v=None):
    """(func(xs), J·v): the Jacobian-vector product; v defaults to ones like the inputs."""
    xl, single = _as_list(xs)
    leaves = [_leaf(x) for x in xl]
    ys = func(*[Tensor(t) for t in leaves])
    yl, ysingle = _as_list(ys)
    yt = [_u(y) for y in yl]
    tangents = [torch.ones_like(x) for x in leaves] if v is None else _check_v(v, leaves, 'jvp')
    ws = [torch.zeros_like(y, requires_grad=True) for y in yt]
    g = _grads(yt, leaves, ws, create_graph=True)
    out = _grads([gi for gi in g], ws, tangents, retain_graph=False) if any(gi.requires_grad for gi in g) \
        else [torch.zeros_like(y) for y in yt]
    out = [Tensor(o) for o in out]
    return ys, (out[0] if ysingle else out)


class _LazyJacobian:
    """Rows of the lazy axis (outputs) computed on demand by reverse passes, cached."""

    def __init__(self, func, xs, is_batched, create_graph=False, detach=True):
        xl, _ = _as_list(xs)
        self._xs = [_leaf(x, keep_graph=not detach) for x in xl]
        ys = func(*[Tensor(t) for t in self._xs])
        yl, _ = _as_list(ys)
        self._batched = is_batched
        self._create_graph = create_graph
        yt = [_u(y) for y in yl]
        if is_batched:
            B = self._xs[0].shape[0]
            for t in self._xs + yt:
                if t.dim() == 0 or t.shape[0] != B:
                    raise ValueError("Jacobian(is_batched=True): every input and output needs the batch "
                                     f"size {B} as its first dimension")
            self._fy = torch.cat([y.reshape(B, -1) for y in yt], 1)
            self._nx = sum(x[0].numel() for x in self._xs)
        else:
            self._fy = torch.cat([y.reshape(-1) for y in yt])
            self._nx = sum(x.numel() for x in self._xs)
        self._cache = {}

    @property
    def shape(self):
        if self._batched:
            return [self._fy.shape[0], self._fy.shape[1], self._nx]
        return [self._fy.shape[0], self._nx]

    def _row(self, k):
        r = self._cache.get(k)
        if r is None:
            if self._batched:
                y = self._fy[:, k]
                gs = _grads([y], self._xs, [torch.ones_like(y)], create_graph=self._create_graph)
                r = torch.cat([g.reshape(g.shape[0], -1) for g in gs], 1)
            else:
                y = self._fy[k]
                gs = _grads([y], self._xs, [torch.ones_like(y)], create_graph=self._create_graph)
                r = torch.cat([g.reshape(-1) for g in gs])
            self._cache[k] = r
        return r

    def __getitem__(self, idx):
        ndim = 3 if self._batched else 2
        if not isinstance(idx, tuple):
            idx = (idx,)
        if any(i is Ellipsis for i in idx):
            p = idx.index(Ellipsis)
            idx = idx[:p] + (slice(None),) * (ndim - len(idx) + 1) + idx[p + 1:]
        if len(idx) > ndim:
            raise IndexError(f"too many indices for a {ndim}-D Jacobian")
        idx = tuple(idx) + (slice(None),) * (ndim - len(idx))
        la = 1 if self._batched else 0
        li = idx[la]
        n = self._fy.shape[la]
        if isinstance(li, slice):
            rows = list(range(n))[li]
        else:
            k = int(li)
            if not -n <= k < n:
                raise IndexError(f"Jacobian index {k} out of range for size {n}")
            rows = [k % n]
        if self._batched:
            return Tensor(self._batched_index(idx, rows, li))
        mats = [self._row(k) for k in rows]
        m = torch.stack(mats, 0) if mats else self._fy.new_zeros((0, self._nx))
        m = m[:, idx[1]]
        if not isinstance(li, slice):
            m = m[0]
        return Tensor(m)

    def _batched_index(self, idx, rows, li):
        # [B][rows][Nx], then each integer index drops its axis
        mats = [self._row(k) for k in rows]
        full = torch.stack(mats, 1) if mats else self._fy.new_zeros((self._fy.shape[0], 0, self._nx))
        out = full[idx[0]] if isinstance(idx[0], slice) else full[int(idx[0])].unsqueeze(0)
        out = out[:, :, idx[2]] if isinstance(idx[2], slice) else out[:, :, int(idx[2])].unsqueeze(2)
        if not isinstance(idx[2], slice):
            out = out.squeeze(2)
        if not isinstance(li, slice):
            out = out.squeeze(1)
        if not isinstance(idx[0], slice):
            out = out.squeeze(0)
        return out


class Jacobian:
    """Lazy Jacobian of ``func`` at ``xs``. Unbatched: shape [numel(ys), numel(xs)] (outputs and
    inputs flattened and concatenated). ``is_batched``: inputs and outputs carry the batch as
    their first axis, shape [B, Ny, Nx] (the function must not mix batch elements)."""

    def __init__(self, func, xs, is_batched=False):
        self._j = _LazyJacobian(func, xs, is_batched)

    def __getitem__(self, idx):
        return self._j[idx]

    @property
    def shape(self):
        return self._j.shape


class Hessian:
    """Lazy Hessian of a scalar-valued ``func`` (batched: [B, 1] outputs) at ``xs``: the Jacobian
    of its gradient, shape [Nx, Nx] or [B, Nx, Nx]."""

    def __init__(self, func, xs, is_batched=False):
        def grad_func(*ts):
            inner = _LazyJacobian(func, ts, is_batched, create_graph=True, detach=False)
            sh = inner.shape
            if (is_batched and sh[1] != 1) or (not is_batched and sh[0] != 1):
                raise RuntimeError("The function given to Hessian should return a single-element Tensor "
                                   "(or a batch of single elements with is_batched=True)")
            row = inner._row(0)
            return Tensor(row)
        self._j = _LazyJacobian(grad_func, xs, is_batched)

    def __getitem__(self, idx):
        return self._j[idx]

    @property
    def shape(self):
        return self._j.shape
