"""paddle.sparse (parity: python/paddle/sparse/*): COO/CSR tensors on PyTorch-ROCm sparse storage.

Unary ops map the stored values (the reference's values-only unary kernels); binary ops, the
products (SpMM / SpGEMM / SDDMM), transpose and reshape compute on the coordinates directly
(sparse/ops.py, sparse/rulebook.py) -- nothing is densified."""
import torch

from ..framework.core import Tensor, _u, convert_dtype, _default_device
from . import ops as _K


def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    i, v = torch.as_tensor(_u(indices)), torch.as_tensor(_u(values))
    if dtype is not None:
        v = v.to(convert_dtype(dtype))
    t = torch.sparse_coo_tensor(i, v, shape, device=_default_device()).coalesce()
    out = Tensor(t)
    out.stop_gradient = stop_gradient
    return out


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    v = torch.as_tensor(_u(values))
    if dtype is not None:
        v = v.to(convert_dtype(dtype))
    return Tensor(torch.sparse_csr_tensor(torch.as_tensor(_u(crows)), torch.as_tensor(_u(cols)),
                                          v, shape, device=_default_device()))


def _vals_op(fn):
    def op(x, *a, name=None):
        t = _u(x)
        if t.layout == torch.sparse_coo:
            t = t.coalesce()
            return Tensor(torch.sparse_coo_tensor(t.indices(), fn(t.values(), *a), t.shape))
        if t.layout == torch.sparse_csr:
            return Tensor(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(),
                                                  fn(t.values(), *a), t.shape))
        return Tensor(fn(t, *a))
    return op


sin, tan, asin, atan, sinh, tanh, asinh, atanh, sqrt, square, log1p, abs, neg, deg2rad, rad2deg, \
    expm1 = (_vals_op(getattr(torch, n)) for n in
             ('sin', 'tan', 'asin', 'atan', 'sinh', 'tanh', 'asinh', 'atanh', 'sqrt', 'square',
              'log1p', 'abs', 'neg', 'deg2rad', 'rad2deg', 'expm1'))
pow = _vals_op(torch.pow)


def cast(x, index_dtype=None, value_dtype=None, name=None):
    return _vals_op(lambda v: v.to(convert_dtype(value_dtype)) if value_dtype else v)(x)


def _sparse(t):
    return t.layout in (torch.sparse_coo, torch.sparse_csr)


def _bin(op, dense_fn):
    def f(x, y, name=None):
        a, b = _u(x), _u(y)
        if _sparse(a) and _sparse(b):
            return Tensor(_K.elementwise(op, a, b))
        if _sparse(a) or _sparse(b):       # mixed: the result is dense, like the reference
            a = a.to_dense() if _sparse(a) else a
            b = b.to_dense() if _sparse(b) else b
        return Tensor(dense_fn(a, b))
    f.__name__ = op
    f.__doc__ = f"Sparse {op}: merged coordinate patterns (sparse/ops.py elementwise)."
    return f


add, subtract, multiply, divide = (_bin(n, f) for n, f in (('add', torch.add), ('subtract', torch.sub),
                                                           ('multiply', torch.mul),
                                                           ('divide', torch.div)))


def matmul(x, y, name=None):
    """sparse @ dense (SpMM), sparse @ sparse (SpGEMM, result in x's layout), dense @ sparse."""
    a, b = _u(x), _u(y)
    if _sparse(a) and _sparse(b):
        return Tensor(_K.spgemm(a, b))
    if _sparse(a):
        return Tensor(_K.spmm(a, b))
    if _sparse(b):
        return Tensor(_K.dense_spmm(a, b))
    return Tensor(torch.matmul(a, b))


def masked_matmul(x, y, mask, name=None):
    """(x @ y) evaluated only at ``mask``'s coordinates (SDDMM); result has mask's layout."""
    return Tensor(_K.sddmm(_u(x), _u(y), _u(mask)))


def mv(x, vec, name=None):
    return Tensor(_K.spmm(_u(x), _u(vec)))


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    """beta * input + alpha * (x @ y); sparse input with sparse x, y stays sparse."""
    inp, prod = _u(input), _u(matmul(x, y))
    if _sparse(inp) and _sparse(prod):
        return Tensor(_K.elementwise('add', _vals_scale(inp, beta), _vals_scale(prod, alpha)))
    inp = inp.to_dense() if _sparse(inp) else inp
    prod = prod.to_dense() if _sparse(prod) else prod
    return Tensor(beta * inp + alpha * prod)


def _vals_scale(t, s):
    idx, v, shape, layout = _K.coo_parts(t)
    return _K.make(idx, v * s, shape, layout, coalesced=True)


def transpose(x, perm, name=None):
    """Permute the sparse dims by permuting the coordinate rows (dense dims stay last)."""
    idx, v, shape, layout = _K.coo_parts(_u(x))
    sd = idx.shape[0]
    perm = [p % len(shape) for p in perm]
    if sorted(perm[:sd]) != list(range(sd)) or perm[sd:] != list(range(sd, len(shape))):
        raise ValueError(f"sparse transpose permutes the sparse dims only; got perm {perm}")
    return Tensor(_K.make(idx[perm[:sd]], v, tuple(shape[p] for p in perm), layout))


def reshape(x, shape, name=None):
    """Reshape the SPARSE dims of a COO tensor without densifying: every index tuple is
    linearised over the old sparse shape and unravelled over the new one (dense trailing dims,
    e.g. channels, must be unchanged). CSR inputs go through COO."""
    t = _u(x)
    csr = t.layout == torch.sparse_csr
    t = (t.to_sparse_coo() if csr else t).coalesce()
    sd, dd = t.sparse_dim(), t.dense_dim()
    old_sp = list(t.shape[:sd])
    dense = list(t.shape[sd:])
    shape = list(shape)
    n_sp = 1
    for v in old_sp:
        n_sp *= v
    if -1 in shape:
        known = 1
        for v in shape:
            if v != -1:
                known *= v
        shape[shape.index(-1)] = (n_sp * max(1, _prod(dense))) // known
    if dd:
        if shape[len(shape) - dd:] != dense:
            raise ValueError(f"sparse reshape keeps the dense dims {dense}; got {shape}")
        new_sp = shape[:len(shape) - dd]
    else:
        new_sp = shape
    if _prod(new_sp) != n_sp:
        raise ValueError(f"cannot reshape sparse dims {old_sp} into {new_sp}")
    idx = t.indices()
    lin = torch.zeros(idx.shape[1], dtype=torch.int64, device=idx.device)
    for d, n in enumerate(old_sp):
        lin = lin * n + idx[d]
    out = []
    for n in reversed(new_sp):
        out.append(lin % n)
        lin = lin // n
    nidx = torch.stack(out[::-1]) if out else idx[:0]
    r = torch.sparse_coo_tensor(nidx, t.values(), new_sp + dense).coalesce()
    return Tensor(r.to_sparse_csr() if csr and len(new_sp) == 2 and not dd else r)


def _prod(v):
    p = 1
    for x in v:
        p *= x
    return p


def coalesce(x, name=None):
    return Tensor(_u(x).coalesce())


def is_same_shape(x, y):
    return list(_u(x).shape) == list(_u(y).shape)


from . import nn  # noqa
