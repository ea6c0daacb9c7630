"""Linear algebra (parity: python/paddle/tensor/linalg.py, python/paddle/linalg.py).

``matmul`` / ``mm`` with a 2-D right operand in bf16/fp16 on the device run the framework GEMM
(``ops.fused.linear`` / ``linear_nt``: the in-tree MFMA kernel through the registry, hipBLASLt
where the shape policy prefers it, autograd through LinearFn / LinearNTFn); batched products and
the factorisations / solvers (inv, det, svd, qr, lu, cholesky, eig*, lstsq, ...) are the
rocSOLVER / hipBLAS-backed torch.linalg routines with Paddle's argument and return conventions
(``slogdet`` stacked [sign, logabsdet], 1-based int32 LU pivots, ``triangular_solve`` transpose
flag, ``norm`` p / axis combinations).
"""
import torch

from ..framework.core import Tensor, _u
from ..amp import amp_op as _amp_op


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


def _gemm_ok(a, b):
    return (a.is_cuda and b.is_cuda and a.dtype == b.dtype and a.dtype in (torch.bfloat16, torch.float16)
            and a.dim() >= 2 and b.dim() == 2)


@_amp_op('matmul')
def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    a, b = _t(x), _t(y)
    if not transpose_x and _gemm_ok(a, b):
        from ..ops import fused as _K
        if transpose_y:
            y2 = _K.linear_nt(a.reshape(-1, a.shape[-1]), b)
            return Tensor(y2.view(*a.shape[:-1], b.shape[0]))
        return Tensor(_K.linear(a, b))
    if transpose_x:
        a = a.transpose(-1, -2) if a.dim() > 1 else a
    if transpose_y:
        b = b.transpose(-1, -2) if b.dim() > 1 else b
    return Tensor(torch.matmul(a, b))


@_amp_op('mm')
def mm(input, mat2, name=None):
    return matmul(input, mat2)


@_amp_op('bmm')
def bmm(x, y, name=None):
    return Tensor(torch.bmm(_t(x), _t(y)))


def mv(x, vec, name=None):
    return Tensor(torch.mv(_t(x), _t(vec)))


def dot(x, y, name=None):
    a, b = _t(x), _t(y)
    if a.dim() == 2:
        return Tensor((a * b).sum(-1))
    return Tensor(torch.dot(a, b))


def cross(x, y, axis=9, name=None):
    a, b = _t(x), _t(y)
    if axis == 9:
        axis = next(i for i, s in enumerate(a.shape) if s == 3)
    return Tensor(torch.linalg.cross(a, b, dim=axis))


def einsum(equation, *operands):
    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = operands[0]
    return Tensor(torch.einsum(equation, *[_t(o) for o in operands]))


def norm(x, p='fro', axis=None, keepdim=False, name=None):
    t = _t(x)
    if isinstance(axis, (list, tuple)) and len(axis) == 1:
        axis = axis[0]
    if p == 'fro':
        if axis is None or isinstance(axis, int):
            return Tensor(torch.linalg.vector_norm(t, 2, dim=axis, keepdim=keepdim))
        return Tensor(torch.linalg.matrix_norm(t, 'fro', dim=tuple(axis), keepdim=keepdim))
    if p == 'nuc':
        return Tensor(torch.linalg.matrix_norm(t, 'nuc', dim=tuple(axis or (-2, -1)),
                                               keepdim=keepdim))
    if isinstance(axis, (list, tuple)) and len(axis) == 2 and p not in (float('inf'), -float('inf'),
                                                                        0):
        return Tensor(torch.linalg.vector_norm(t, float(p), dim=tuple(axis), keepdim=keepdim))
    return Tensor(torch.linalg.vector_norm(t, float(p), dim=axis, keepdim=keepdim))


def vector_norm(x, p=2.0, axis=None, keepdim=False, name=None):
    return Tensor(torch.linalg.vector_norm(_t(x), p, dim=axis, keepdim=keepdim))


def matrix_norm(x, p='fro', axis=[-2, -1], keepdim=False, name=None):
    return Tensor(torch.linalg.matrix_norm(_t(x), p, dim=tuple(axis), keepdim=keepdim))


def cond(x, p=None, name=None):
    return Tensor(torch.linalg.cond(_t(x), p))


def cov(x, rowvar=True, ddof=True, fweights=None, aweights=None, name=None):
    t = _t(x)
    if not rowvar:
        t = t.t()
    return Tensor(torch.cov(t, correction=1 if ddof else 0,
                            fweights=None if fweights is None else _t(fweights),
                            aweights=None if aweights is None else _t(aweights)))


def corrcoef(x, rowvar=True, name=None):
    t = _t(x)
    return Tensor(torch.corrcoef(t if rowvar else t.t()))


def inv(x, name=None):
    return Tensor(torch.linalg.inv(_t(x)))


def det(x, name=None):
    return Tensor(torch.linalg.det(_t(x)))


def slogdet(x, name=None):
    s, l = torch.linalg.slogdet(_t(x))
    return Tensor(torch.stack([s, l]))


def eig(x, name=None):
    w, v = torch.linalg.eig(_t(x))
    return Tensor(w), Tensor(v)


def eigvals(x, name=None):
    return Tensor(torch.linalg.eigvals(_t(x)))


def eigh(x, UPLO='L', name=None):
    w, v = torch.linalg.eigh(_t(x), UPLO)
    return Tensor(w), Tensor(v)


def eigvalsh(x, UPLO='L', name=None):
    return Tensor(torch.linalg.eigvalsh(_t(x), UPLO))


def svd(x, full_matrices=False, name=None):
    u, s, vh = torch.linalg.svd(_t(x), full_matrices=full_matrices)
    return Tensor(u), Tensor(s), Tensor(vh)


def qr(x, mode='reduced', name=None):
    q, r = torch.linalg.qr(_t(x), mode)
    if mode == 'r':
        return Tensor(r)
    return Tensor(q), Tensor(r)


def lu(x, pivot=True, get_infos=False, name=None):
    lu_, piv = torch.linalg.lu_factor(_t(x), pivot=pivot)
    piv = piv.to(torch.int32)
    if get_infos:
        return Tensor(lu_), Tensor(piv), Tensor(torch.zeros(lu_.shape[:-2], dtype=torch.int32))
    return Tensor(lu_), Tensor(piv)


def lu_unpack(x, y, unpack_ludata=True, unpack_pivots=True, name=None):
    p, l, u = torch.lu_unpack(_t(x), _t(y))
    return Tensor(p), Tensor(l), Tensor(u)


def cholesky(x, upper=False, name=None):
    return Tensor(torch.linalg.cholesky(_t(x), upper=upper))


def cholesky_solve(x, y, upper=False, name=None):
    return Tensor(torch.cholesky_solve(_t(x), _t(y), upper))


def solve(x, y, name=None):
    return Tensor(torch.linalg.solve(_t(x), _t(y)))


def triangular_solve(x, y, upper=True, transpose=False, unitriangular=False, name=None):
    a = _t(x)
    if transpose:
        a = a.transpose(-1, -2)
        upper = not upper
    return Tensor(torch.linalg.solve_triangular(a, _t(y), upper=upper,
                                                unitriangular=unitriangular))


def lstsq(x, y, rcond=None, driver=None, name=None):
    r = torch.linalg.lstsq(_t(x), _t(y), rcond=rcond, driver=driver)
    return Tensor(r.solution), Tensor(r.residuals), Tensor(r.rank), Tensor(r.singular_values)


def matrix_rank(x, tol=None, hermitian=False, name=None):
    return Tensor(torch.linalg.matrix_rank(_t(x), atol=tol, hermitian=hermitian))


def matrix_power(x, n, name=None):
    return Tensor(torch.linalg.matrix_power(_t(x), n))


def multi_dot(x, name=None):
    return Tensor(torch.linalg.multi_dot([_t(e) for e in x]))


def pinv(x, rcond=1e-15, hermitian=False, name=None):
    return Tensor(torch.linalg.pinv(_t(x), rtol=rcond, hermitian=hermitian))


def matrix_exp(x, name=None):
    return Tensor(torch.linalg.matrix_exp(_t(x)))


def histogramdd(x, bins=10, ranges=None, density=False, weights=None, name=None):
    """D-dimensional histogram of the points x[..., D] -> (hist, [edges per dim])."""
    t = _t(x)
    pts = t.reshape(-1, t.shape[-1]).double().cpu()
    w = None if weights is None else _t(weights).reshape(-1).double().cpu()
    if isinstance(bins, (list, tuple)) and bins and not isinstance(bins[0], int):
        b = [_t(e).double().cpu() if isinstance(e, Tensor) else torch.as_tensor(e, dtype=torch.float64)
             for e in bins]
        hist, edges = torch.histogramdd(pts, bins=b, weight=w, density=density)
    else:
        rg = None if ranges is None else [float(r) for r in ranges]
        hist, edges = torch.histogramdd(pts, bins=bins, range=rg, weight=w, density=density)
    return Tensor(hist.to(t.dtype if t.is_floating_point() else torch.float32).to(t.device)), \
        [Tensor(e.to(t.dtype if t.is_floating_point() else torch.float32).to(t.device)) for e in edges]
