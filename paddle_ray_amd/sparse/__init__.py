"""paddle.sparse (parity: python/paddle/sparse/*): COO/CSR tensors on PyTorch-ROCm sparse storage."""
import torch

from ..framework.core import Tensor, _u, convert_dtype, _default_device


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


def _bin(fn):
    def op(x, y, name=None):
        return Tensor(fn(_u(x), _u(y)))
    return op


add, subtract, multiply, divide = _bin(torch.add), _bin(torch.sub), _bin(torch.mul), \
    _bin(torch.div)


def matmul(x, y, name=None):
    return Tensor(torch.sparse.mm(_u(x), _u(y)) if _u(x).is_sparse else torch.matmul(_u(x), _u(y)))


def masked_matmul(x, y, mask, name=None):
    return Tensor(torch.sparse.sampled_addmm(_u(mask).to_sparse_csr(), _u(x), _u(y),
                                             beta=0.0))


def mv(x, vec, name=None):
    return Tensor(torch.mv(_u(x), _u(vec)))


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    return Tensor(torch.sparse.addmm(_u(input), _u(x), _u(y), beta=beta, alpha=alpha))


def transpose(x, perm, name=None):
    return Tensor(_u(x).permute(*perm))


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
