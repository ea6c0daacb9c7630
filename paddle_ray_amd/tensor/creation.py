"""Tensor creation API (parity: python/paddle/tensor/creation.py)."""
import numpy as np
import torch

from ..framework.core import (Tensor, _u, _w, convert_dtype, get_default_dtype, _to_torch_device,
                              to_tensor, _default_device, Parameter)


def _dt(dtype, default=None):
    d = convert_dtype(dtype)
    return d if d is not None else (default if default is not None else get_default_dtype())


def _shape(shape):
    if isinstance(shape, Tensor):
        return [int(v) for v in shape._t.tolist()]
    if isinstance(shape, (int, np.integer)):
        return [int(shape)]
    return [int(s.item()) if isinstance(s, Tensor) else int(s) for s in shape]


def _dev():
    return _default_device()


def create_tensor(dtype, name=None, persistable=False):
    """An empty tensor of ``dtype`` to be filled later, e.g. by ``paddle.assign`` (parity:
    python/paddle/tensor/creation.py create_tensor; dygraph form: shape [0])."""
    t = zeros([0], dtype=dtype)
    t.persistable = bool(persistable)
    if name is not None:
        t.name = name
    return t


def zeros(shape, dtype=None, name=None):
    return Tensor(torch.zeros(_shape(shape), dtype=_dt(dtype), device=_dev()))


def ones(shape, dtype=None, name=None):
    return Tensor(torch.ones(_shape(shape), dtype=_dt(dtype), device=_dev()))


def empty(shape, dtype=None, name=None):
    return Tensor(torch.empty(_shape(shape), dtype=_dt(dtype), device=_dev()))


def full(shape, fill_value, dtype=None, name=None):
    if isinstance(fill_value, Tensor):
        fill_value = fill_value.item()
    if dtype is None:
        dtype = torch.bool if isinstance(fill_value, bool) else get_default_dtype()
    return Tensor(torch.full(_shape(shape), fill_value, dtype=_dt(dtype), device=_dev()))


def zeros_like(x, dtype=None, name=None):
    t = _u(x)
    return Tensor(torch.zeros_like(t, dtype=convert_dtype(dtype) or t.dtype))


def ones_like(x, dtype=None, name=None):
    t = _u(x)
    return Tensor(torch.ones_like(t, dtype=convert_dtype(dtype) or t.dtype))


def empty_like(x, dtype=None, name=None):
    t = _u(x)
    return Tensor(torch.empty_like(t, dtype=convert_dtype(dtype) or t.dtype))


def full_like(x, fill_value, dtype=None, name=None):
    t = _u(x)
    return Tensor(torch.full_like(t, fill_value, dtype=convert_dtype(dtype) or t.dtype))


def arange(start=0, end=None, step=1, dtype=None, name=None):
    start, end, step = [v.item() if isinstance(v, Tensor) else v for v in (start, end, step)]
    if end is None:
        start, end = 0, start
    if dtype is None:
        dtype = torch.int64 if all(isinstance(v, (int, np.integer)) for v in (start, end, step)) \
            else get_default_dtype()
    return Tensor(torch.arange(start, end, step, dtype=convert_dtype(dtype), device=_dev()))


def linspace(start, stop, num, dtype=None, name=None):
    start, stop, num = [v.item() if isinstance(v, Tensor) else v for v in (start, stop, num)]
    return Tensor(torch.linspace(start, stop, int(num), dtype=_dt(dtype), device=_dev()))


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    return Tensor(torch.logspace(float(start), float(stop), int(num), base=float(base),
                                 dtype=_dt(dtype), device=_dev()))


def eye(num_rows, num_columns=None, dtype=None, name=None):
    num_columns = num_rows if num_columns is None else num_columns
    return Tensor(torch.eye(int(num_rows), int(num_columns), dtype=_dt(dtype), device=_dev()))


def diag(x, offset=0, padding_value=0, name=None):
    t = _u(x)
    if t.dim() == 1 and padding_value != 0:
        n = t.shape[0] + abs(offset)
        out = torch.full((n, n), padding_value, dtype=t.dtype, device=t.device)
        return Tensor(out + torch.diag(t, offset) - torch.diag(torch.full_like(t, padding_value), offset))
    return Tensor(torch.diag(t, offset))


def diagflat(x, offset=0, name=None):
    return Tensor(torch.diagflat(_u(x), offset))


def diag_embed(input, offset=0, dim1=-2, dim2=-1):
    return Tensor(torch.diag_embed(_u(input), offset, dim1, dim2))


def tril(x, diagonal=0, name=None):
    return Tensor(torch.tril(_u(x), diagonal))


def triu(x, diagonal=0, name=None):
    return Tensor(torch.triu(_u(x), diagonal))


def tril_indices(row, col, offset=0, dtype='int64'):
    return Tensor(torch.tril_indices(row, col, offset, dtype=convert_dtype(dtype), device=_dev()))


def triu_indices(row, col=None, offset=0, dtype='int64'):
    col = row if col is None else col
    return Tensor(torch.triu_indices(row, col, offset, dtype=convert_dtype(dtype), device=_dev()))


def meshgrid(*args, **kwargs):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return [Tensor(t) for t in torch.meshgrid(*[_u(a) for a in args], indexing='ij')]


def assign(x, output=None):
    if isinstance(x, Tensor):
        t = x._t.clone()
    else:
        t = torch.as_tensor(np.asarray(x), device=_dev())
        if t.dtype == torch.float64 and not isinstance(x, np.ndarray):
            t = t.to(get_default_dtype())
    if output is not None:
        with torch.no_grad():
            if output._t.shape != t.shape and output._t.numel() == 0:
                # an empty placeholder (create_tensor): takes the value's shape, keeps its dtype
                output._t.set_(t.to(output._t.dtype).contiguous())
            else:
                output._t.copy_(t)
        return output
    return Tensor(t)


def clone(x, name=None):
    return Tensor(_u(x).clone())


def complex(real, imag, name=None):
    return Tensor(torch.complex(_u(real), _u(imag)))


def polar(abs, angle, name=None):
    return Tensor(torch.polar(_u(abs), _u(angle)))


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..nn.initializer import _init_param
    p = Parameter(torch.empty(_shape(shape), dtype=convert_dtype(dtype), device=_dev()), name=name)
    _init_param(p, attr, default_initializer, is_bias)
    return p


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    t = full(shape, value, dtype)
    t.persistable = persistable
    return t
