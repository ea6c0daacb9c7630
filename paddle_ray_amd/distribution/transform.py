"""Bijective / injective transforms for TransformedDistribution (parity:
python/paddle/distribution/transform.py): forward / inverse maps, their log|det J|, the shapes
they map, and the event rank each one consumes (``_event_rank_in``) and produces
(``_event_rank``). Written out as tensor math (no torch.distributions objects)."""
import enum
import math

import torch
import torch.nn.functional as TF

from ..framework.core import Tensor, _u

__all__ = ['Transform', 'AbsTransform', 'AffineTransform', 'ChainTransform', 'ExpTransform',
           'IndependentTransform', 'PowerTransform', 'ReshapeTransform', 'SigmoidTransform',
           'SoftmaxTransform', 'StackTransform', 'StickBreakingTransform', 'TanhTransform']


class Type(enum.Enum):
    BIJECTION = 'bijection'
    INJECTION = 'injection'
    SURJECTION = 'surjection'
    OTHER = 'other'

    @classmethod
    def is_injective(cls, t):
        return t in (cls.BIJECTION, cls.INJECTION)


def _v(x):
    if isinstance(x, Tensor):
        return x._t
    t = torch.as_tensor(x)
    return t if t.is_floating_point() else t.to(torch.get_default_dtype())


def _sum_right(t, n):
    return t.sum(tuple(range(-n, 0))) if n > 0 else t


class Transform:
    """y = f(x). Subclasses implement ``_fwd``, ``_inv`` and ``_fldj`` (log|det df/dx|, reduced
    over the ``_event_rank_in`` rightmost dims of x)."""
    _type = Type.BIJECTION
    _event_rank_in = 0
    _event_rank = 0

    @classmethod
    def _is_injective(cls):
        return Type.is_injective(cls._type)

    def __call__(self, x):
        from .distribution import Distribution, TransformedDistribution
        if isinstance(x, Distribution):
            return TransformedDistribution(x, [self])
        if isinstance(x, Transform):
            return ChainTransform([x, self])
        return self.forward(x)

    def forward(self, x):
        return Tensor(self._fwd(_v(x)))

    def inverse(self, y):
        return Tensor(self._inv(_v(y)))

    def forward_log_det_jacobian(self, x):
        return Tensor(self._fldj(_v(x)))

    def inverse_log_det_jacobian(self, y):
        y = _v(y)
        return Tensor(-self._fldj(self._inv(y)))

    def forward_shape(self, shape):
        return list(shape)

    def inverse_shape(self, shape):
        return list(shape)

    def _fwd(self, x):
        raise NotImplementedError

    def _inv(self, y):
        raise NotImplementedError

    def _fldj(self, x):
        raise NotImplementedError


class AbsTransform(Transform):
    """y = |x| (surjective): inverse returns the two preimages (-y, y)."""
    _type = Type.SURJECTION

    def _fwd(self, x):
        return x.abs()

    def inverse(self, y):
        y = _v(y)
        return Tensor(-y), Tensor(y)

    def _inv(self, y):
        return y

    def _fldj(self, x):
        return torch.zeros_like(x)

    def inverse_log_det_jacobian(self, y):
        z = torch.zeros_like(_v(y))
        return Tensor(z), Tensor(z)


class AffineTransform(Transform):
    """y = loc + scale * x."""

    def __init__(self, loc, scale):
        self.loc, self.scale = loc, scale
        self._loc, self._scale = _v(loc), _v(scale)

    def _fwd(self, x):
        return self._loc.to(x) + self._scale.to(x) * x

    def _inv(self, y):
        return (y - self._loc.to(y)) / self._scale.to(y)

    def _fldj(self, x):
        return torch.broadcast_to(self._scale.to(x).abs().log(), torch.broadcast_shapes(x.shape, self._scale.shape))

    def forward_shape(self, shape):
        return list(torch.broadcast_shapes(tuple(shape), self._loc.shape, self._scale.shape))

    inverse_shape = forward_shape


class ExpTransform(Transform):
    """y = exp(x), log|dy/dx| = x."""

    def _fwd(self, x):
        return x.exp()

    def _inv(self, y):
        return y.log()

    def _fldj(self, x):
        return x


class PowerTransform(Transform):
    """y = x ** power on x > 0."""

    def __init__(self, power):
        self.power = power
        self._p = _v(power)

    def _fwd(self, x):
        return x.pow(self._p.to(x))

    def _inv(self, y):
        return y.pow(1.0 / self._p.to(y))

    def _fldj(self, x):
        p = self._p.to(x)
        return (p * x.pow(p - 1)).abs().log()

    def forward_shape(self, shape):
        return list(torch.broadcast_shapes(tuple(shape), self._p.shape))

    inverse_shape = forward_shape


class SigmoidTransform(Transform):
    """y = 1 / (1 + exp(-x)), log|dy/dx| = -softplus(-x) - softplus(x)."""

    def _fwd(self, x):
        return torch.sigmoid(x)

    def _inv(self, y):
        return y.log() - (-y).log1p()

    def _fldj(self, x):
        return -TF.softplus(-x) - TF.softplus(x)


class TanhTransform(Transform):
    """y = tanh(x), log|dy/dx| = 2 (log 2 - x - softplus(-2x)) (stable form of log(1 - tanh^2))."""

    def _fwd(self, x):
        return torch.tanh(x)

    def _inv(self, y):
        return torch.atanh(y)

    def _fldj(self, x):
        return 2.0 * (math.log(2.0) - x - TF.softplus(-2.0 * x))


class SoftmaxTransform(Transform):
    """y = softmax(x) over the last dim (not injective: inverse is log y, up to a constant)."""
    _type = Type.OTHER
    _event_rank_in = 1
    _event_rank = 1

    def _fwd(self, x):
        return torch.softmax(x, -1)

    def _inv(self, y):
        return y.log()

    def _fldj(self, x):
        raise NotImplementedError("SoftmaxTransform is not injective")


class StickBreakingTransform(Transform):
    """R^(K-1) -> the K-simplex: z_i = sigmoid(x_i - log(K-1-i)), y_i = z_i * prod_{j<i}(1 - z_j),
    y_K = prod_j (1 - z_j)."""
    _event_rank_in = 1
    _event_rank = 1

    def _fwd(self, x):
        n = x.shape[-1]
        off = torch.log(torch.arange(n, 0, -1, dtype=x.dtype, device=x.device))
        z = torch.sigmoid(x - off)
        rest = torch.cumprod(1 - z, -1)
        y = torch.cat([z, torch.ones_like(z[..., :1])], -1)
        y = y * torch.cat([torch.ones_like(z[..., :1]), rest], -1)
        return y

    def _inv(self, y):
        n = y.shape[-1] - 1
        off = torch.log(torch.arange(n, 0, -1, dtype=y.dtype, device=y.device))
        rem = 1 - torch.cumsum(y[..., :-1], -1)
        rem = torch.cat([torch.ones_like(y[..., :1]), rem[..., :-1]], -1)
        z = y[..., :-1] / rem
        return z.log() - (-z).log1p() + off

    def _fldj(self, x):
        n = x.shape[-1]
        off = torch.log(torch.arange(n, 0, -1, dtype=x.dtype, device=x.device))
        t = x - off
        z = torch.sigmoid(t)
        # dy_i/dx_i = z_i (1 - z_i) prod_{j<i} (1 - z_j): triangular Jacobian
        log_rest = torch.cumsum(torch.log1p(-z), -1)
        log_rest = torch.cat([torch.zeros_like(z[..., :1]), log_rest[..., :-1]], -1)
        return (-TF.softplus(-t) - TF.softplus(t) + log_rest).sum(-1)

    def forward_shape(self, shape):
        return list(shape[:-1]) + [shape[-1] + 1]

    def inverse_shape(self, shape):
        return list(shape[:-1]) + [shape[-1] - 1]


class ReshapeTransform(Transform):
    """Reshapes the event part: in_event_shape -> out_event_shape (same size)."""

    def __init__(self, in_event_shape, out_event_shape):
        if math.prod(in_event_shape) != math.prod(out_event_shape):
            raise ValueError("in_event_shape and out_event_shape must have the same size")
        self.in_event_shape, self.out_event_shape = tuple(in_event_shape), tuple(out_event_shape)
        self._event_rank_in, self._event_rank = len(self.in_event_shape), len(self.out_event_shape)

    def _fwd(self, x):
        b = x.shape[:x.dim() - len(self.in_event_shape)]
        return x.reshape(tuple(b) + self.out_event_shape)

    def _inv(self, y):
        b = y.shape[:y.dim() - len(self.out_event_shape)]
        return y.reshape(tuple(b) + self.in_event_shape)

    def _fldj(self, x):
        return x.new_zeros(x.shape[:x.dim() - len(self.in_event_shape)])

    def forward_shape(self, shape):
        k = len(self.in_event_shape)
        if tuple(shape[len(shape) - k:]) != self.in_event_shape:
            raise ValueError(f"shape {list(shape)} does not end with {list(self.in_event_shape)}")
        return list(shape[:len(shape) - k]) + list(self.out_event_shape)

    def inverse_shape(self, shape):
        k = len(self.out_event_shape)
        if tuple(shape[len(shape) - k:]) != self.out_event_shape:
            raise ValueError(f"shape {list(shape)} does not end with {list(self.out_event_shape)}")
        return list(shape[:len(shape) - k]) + list(self.in_event_shape)


class ChainTransform(Transform):
    """T_n o ... o T_1; log|det J| adds up over the chain (each term summed over the event dims
    the chain as a whole consumes)."""

    def __init__(self, transforms):
        self.transforms = list(transforms)
        # event ranks of the composition: walk the codomain backwards / the domain forwards
        r = self.transforms[-1]._event_rank if self.transforms else 0
        for t in reversed(self.transforms):
            r = max(r + t._event_rank_in - t._event_rank, t._event_rank_in)
        self._event_rank_in = r
        r = self.transforms[0]._event_rank_in if self.transforms else 0
        for t in self.transforms:
            r = max(r + t._event_rank - t._event_rank_in, t._event_rank)
        self._event_rank = r

    @property
    def _type(self):
        return Type.BIJECTION if all(t._is_injective() for t in self.transforms) else Type.OTHER

    def _fwd(self, x):
        for t in self.transforms:
            x = t._fwd(x)
        return x

    def _inv(self, y):
        for t in reversed(self.transforms):
            y = t._inv(y)
        return y

    def _fldj(self, x):
        nd = x.dim() - self._event_rank_in
        total = 0.0
        for t in self.transforms:
            ld = t._fldj(x)
            total = total + _sum_right(ld, ld.dim() - nd)
            x = t._fwd(x)
        if not isinstance(total, torch.Tensor):
            total = x.new_zeros(x.shape[:nd])
        return total

    def forward_shape(self, shape):
        for t in self.transforms:
            shape = t.forward_shape(shape)
        return list(shape)

    def inverse_shape(self, shape):
        for t in reversed(self.transforms):
            shape = t.inverse_shape(shape)
        return list(shape)


class IndependentTransform(Transform):
    """``base`` with its rightmost ``reinterpreted_batch_rank`` dims treated as event dims: the
    log-det is summed over them."""

    def __init__(self, base, reinterpreted_batch_rank):
        if reinterpreted_batch_rank <= 0:
            raise ValueError("reinterpreted_batch_rank must be positive")
        self.base, self.reinterpreted_batch_rank = base, reinterpreted_batch_rank
        self._event_rank_in = base._event_rank_in + reinterpreted_batch_rank
        self._event_rank = base._event_rank + reinterpreted_batch_rank

    @property
    def _type(self):
        return self.base._type

    def _fwd(self, x):
        return self.base._fwd(x)

    def _inv(self, y):
        return self.base._inv(y)

    def _fldj(self, x):
        return _sum_right(self.base._fldj(x), self.reinterpreted_batch_rank)

    def forward_shape(self, shape):
        return self.base.forward_shape(shape)

    def inverse_shape(self, shape):
        return self.base.inverse_shape(shape)


class StackTransform(Transform):
    """Applies ``transforms[i]`` to slice i of ``axis``."""

    def __init__(self, transforms, axis=0):
        if not transforms:
            raise ValueError("StackTransform needs at least one transform")
        self.transforms, self.axis = list(transforms), axis

    def _map(self, x, fn):
        parts = torch.unbind(x, self.axis)
        if len(parts) != len(self.transforms):
            raise ValueError(f"axis {self.axis} has {len(parts)} slices for {len(self.transforms)} transforms")
        return torch.stack([fn(t, p) for t, p in zip(self.transforms, parts)], self.axis)

    def _fwd(self, x):
        return self._map(x, lambda t, p: t._fwd(p))

    def _inv(self, y):
        return self._map(y, lambda t, p: t._inv(p))

    def _fldj(self, x):
        return self._map(x, lambda t, p: t._fldj(p))
