"""paddle.tensor namespace + Tensor method/operator binding.

Parity: python/paddle/tensor/__init__.py (``tensor_method_func`` list) and
python/paddle/fluid/dygraph/math_op_patch.py (operator overloads).
"""
import torch

from ..framework.core import Tensor, _u
from .creation import *  # noqa
from .math import *  # noqa
from .manipulation import *  # noqa
from .linalg import *  # noqa
from .random import *  # noqa
from . import creation, math, manipulation, linalg, random  # noqa

_METHOD_SOURCES = (creation, math, manipulation, linalg, random)
_SKIP = {'seed', 'get_rng_state', 'set_rng_state', 'get_cuda_rng_state', 'set_cuda_rng_state',
         'rand', 'randn', 'randint', 'randperm', 'uniform', 'normal', 'gaussian', 'standard_normal',
         'zeros', 'ones', 'empty', 'full', 'arange', 'linspace', 'logspace', 'eye', 'meshgrid',
         'tril_indices', 'triu_indices', 'create_parameter', 'create_global_var', 'broadcast_shape',
         'complex', 'polar', 'is_tensor', 'builtins_slice'}
_KEEP = {'numel', 'clone', 'tolist', 'cast', 'dim', 'T', 'shape'}


def _bind_methods():
    for mod in _METHOD_SOURCES:
        for name in dir(mod):
            if name.startswith('_') or name in _SKIP:
                continue
            fn = getattr(mod, name)
            if not callable(fn) or isinstance(fn, type):
                continue
            if getattr(fn, '__module__', '').startswith('torch') or name in ('np', 'torch'):
                continue
            if name in Tensor.__dict__ and name not in _KEEP:
                continue
            if name in _KEEP and name in Tensor.__dict__:
                continue
            setattr(Tensor, name, fn)


_bind_methods()


def _binop(fn, reverse=False):
    if reverse:
        def op(self, other):
            o = other._t if isinstance(other, Tensor) else other
            return Tensor(fn(o, self._t) if isinstance(o, torch.Tensor)
                          else fn(torch.as_tensor(o, dtype=_scalar_dtype(self._t, o),
                                                  device=self._t.device), self._t))
    else:
        def op(self, other):
            o = other._t if isinstance(other, Tensor) else other
            if not isinstance(o, (torch.Tensor, int, float, bool, complex)):
                o = torch.as_tensor(o, device=self._t.device)
            return Tensor(fn(self._t, o))
    return op


def _scalar_dtype(t, o):
    if isinstance(o, bool):
        return torch.bool if t.dtype == torch.bool else t.dtype
    if isinstance(o, int):
        return t.dtype
    if isinstance(o, float):
        return t.dtype if t.is_floating_point() else torch.float32
    return None


def _div(a, b):
    return torch.div(a, b)


def _floordiv(a, b):
    return torch.div(a, b, rounding_mode='floor')


def _matmul(a, b):
    return torch.matmul(a, b)


Tensor.__add__ = _binop(torch.add)
Tensor.__radd__ = _binop(torch.add)
Tensor.__sub__ = _binop(torch.sub)
Tensor.__rsub__ = _binop(torch.sub, True)
Tensor.__mul__ = _binop(torch.mul)
Tensor.__rmul__ = _binop(torch.mul)
Tensor.__truediv__ = _binop(_div)
Tensor.__rtruediv__ = _binop(_div, True)
Tensor.__floordiv__ = _binop(_floordiv)
Tensor.__rfloordiv__ = _binop(_floordiv, True)
Tensor.__mod__ = _binop(torch.remainder)
Tensor.__rmod__ = _binop(torch.remainder, True)
Tensor.__pow__ = _binop(torch.pow)
Tensor.__rpow__ = _binop(torch.pow, True)
Tensor.__matmul__ = _binop(_matmul)
Tensor.__rmatmul__ = _binop(_matmul, True)
Tensor.__and__ = _binop(torch.bitwise_and)
Tensor.__or__ = _binop(torch.bitwise_or)
Tensor.__xor__ = _binop(torch.bitwise_xor)
Tensor.__lshift__ = _binop(torch.bitwise_left_shift)
Tensor.__rshift__ = _binop(torch.bitwise_right_shift)
Tensor.__eq__ = _binop(torch.eq)
Tensor.__ne__ = _binop(torch.ne)
Tensor.__lt__ = _binop(torch.lt)
Tensor.__le__ = _binop(torch.le)
Tensor.__gt__ = _binop(torch.gt)
Tensor.__ge__ = _binop(torch.ge)
Tensor.__neg__ = lambda self: Tensor(-self._t)
Tensor.__pos__ = lambda self: self
Tensor.__abs__ = lambda self: Tensor(self._t.abs())
Tensor.__invert__ = lambda self: Tensor(~self._t)


def _iop(name):
    def op(self, other):
        o = other._t if isinstance(other, Tensor) else other
        getattr(self._t, name)(o)
        return self
    return op


Tensor.__iadd__ = _iop('add_')
Tensor.__isub__ = _iop('sub_')
Tensor.__imul__ = _iop('mul_')
Tensor.__itruediv__ = _iop('div_')

# paddle-style method aliases that differ from the functional names
Tensor.add_ = math.add_
Tensor.subtract_ = math.subtract_
Tensor.multiply_ = math.multiply_
Tensor.scale_ = math.scale_
Tensor.clip_ = math.clip_
Tensor.fill_ = math.fill_
Tensor.zero_ = math.zero_
Tensor.uniform_ = random.uniform_
Tensor.normal_ = random.normal_
Tensor.exponential_ = random.exponential_
Tensor.reshape_ = manipulation.reshape_
Tensor.squeeze_ = manipulation.squeeze_
Tensor.unsqueeze_ = manipulation.unsqueeze_
Tensor.flatten_ = manipulation.flatten_
Tensor.scatter_ = manipulation.scatter_
Tensor.numel = lambda self: Tensor(torch.tensor(self._t.numel(), dtype=torch.int64))
Tensor.mm = linalg.mm
Tensor.matmul = linalg.matmul
Tensor.norm = linalg.norm
Tensor.dist = math.dist
Tensor.sum = math.sum
Tensor.mean = math.mean
Tensor.max = math.max
Tensor.min = math.min
Tensor.tolist = lambda self: self._t.tolist()
Tensor.expand = manipulation.expand
Tensor.tile = manipulation.tile
Tensor.split = manipulation.split
Tensor.chunk = manipulation.chunk
Tensor.transpose = manipulation.transpose
Tensor.reshape = manipulation.reshape
Tensor.flatten = manipulation.flatten
Tensor.squeeze = manipulation.squeeze
Tensor.unsqueeze = manipulation.unsqueeze
Tensor.gather = manipulation.gather
Tensor.astype = lambda self, dtype: manipulation.cast(self, dtype)
Tensor.cast = Tensor.astype
Tensor.abs = math.abs
Tensor.sqrt = math.sqrt
Tensor.exp = math.exp
Tensor.log = math.log
Tensor.pow = math.pow
Tensor.sigmoid = math.sigmoid
Tensor.tanh = math.tanh
Tensor.argmax = math.argmax
Tensor.argmin = math.argmin
Tensor.topk = math.topk
Tensor.sort = math.sort
Tensor.argsort = math.argsort
Tensor.where = lambda self, x=None, y=None: math.where(self, x, y)
Tensor.all = math.all
Tensor.any = math.any
Tensor.isnan = math.isnan
Tensor.clip = math.clip
Tensor.equal = math.equal
Tensor.var = math.var
Tensor.std = math.std
Tensor.cumsum = math.cumsum
Tensor.prod = math.prod
Tensor.unbind = manipulation.unbind
Tensor.flip = manipulation.flip
Tensor.roll = manipulation.roll
Tensor.index_select = manipulation.index_select
Tensor.masked_fill = lambda self, mask, value: Tensor(
    self._t.masked_fill(_u(mask), _u(value)))
Tensor.masked_select = math.masked_select
Tensor.broadcast_to = manipulation.broadcast_to
Tensor.expand_as = manipulation.expand_as
Tensor.repeat_interleave = manipulation.repeat_interleave
Tensor.bmm = linalg.bmm
Tensor.dot = linalg.dot
Tensor.t = manipulation.t
Tensor.moveaxis = manipulation.moveaxis
Tensor.diagonal = math.diagonal
Tensor.trace = math.trace
Tensor.logsumexp = math.logsumexp
Tensor.square = math.square
Tensor.rsqrt = math.rsqrt
Tensor.floor = math.floor
Tensor.ceil = math.ceil
Tensor.round = math.round
Tensor.sign = math.sign
Tensor.neg = math.neg
Tensor.reciprocal = math.reciprocal
Tensor.erf = math.erf
Tensor.sin = math.sin
Tensor.cos = math.cos
Tensor.add = math.add
Tensor.subtract = math.subtract
Tensor.multiply = math.multiply
Tensor.divide = math.divide
Tensor.maximum = math.maximum
Tensor.minimum = math.minimum
Tensor.logical_not = math.logical_not
Tensor.logical_and = math.logical_and
Tensor.logical_or = math.logical_or
Tensor.nonzero = math.nonzero
Tensor.unique = math.unique
Tensor.is_floating_point = math.is_floating_point
Tensor.is_complex = math.is_complex
Tensor.slice = manipulation.slice
Tensor.concat = lambda self, others, axis=0: manipulation.concat([self] + list(others), axis)
Tensor.lerp = math.lerp
Tensor.scale = math.scale
Tensor.allclose = math.allclose
Tensor.isclose = math.isclose
Tensor.isinf = math.isinf
Tensor.isfinite = math.isfinite
Tensor.median = math.median
Tensor.quantile = math.quantile
Tensor.nansum = math.nansum
Tensor.amax = math.amax
Tensor.amin = math.amin
Tensor.kron = math.kron
Tensor.inner = math.inner
Tensor.outer = math.outer
Tensor.take_along_axis = manipulation.take_along_axis
Tensor.put_along_axis = manipulation.put_along_axis
Tensor.scatter = manipulation.scatter
Tensor.scatter_nd_add = manipulation.scatter_nd_add
Tensor.gather_nd = manipulation.gather_nd
Tensor.stack = lambda self, others, axis=0: manipulation.stack([self] + list(others), axis)
Tensor.view = manipulation.view
Tensor.tril = creation.tril
Tensor.triu = creation.triu
Tensor.cross = linalg.cross
Tensor.cholesky = linalg.cholesky
Tensor.inverse = linalg.inv
Tensor.remainder = math.remainder
Tensor.mod = math.remainder
Tensor.floor_divide = math.floor_divide
Tensor.floor_mod = math.remainder
Tensor.exp_ = math.exp_
Tensor.erfinv_ = math.erfinv_
Tensor.remainder_ = math.remainder_
Tensor.lerp_ = math.lerp_
Tensor.put_along_axis_ = manipulation.put_along_axis_
Tensor.sqrt_ = math.sqrt_
Tensor.tanh_ = math.tanh_
Tensor.sigmoid_ = math.sigmoid_
Tensor.abs_ = math.abs_
Tensor.neg_ = math.neg_
Tensor.ceil_ = math.ceil_
Tensor.floor_ = math.floor_
Tensor.round_ = math.round_
Tensor.reciprocal_ = math.reciprocal_
Tensor.rsqrt_ = math.rsqrt_
