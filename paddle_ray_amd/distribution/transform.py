"""Bijective / injective transforms for TransformedDistribution (parity:
python/paddle/distribution/transform.py). Each transform wraps the matching
torch.distributions transform (``_t``) and exposes the reference API."""
import enum
import math

import torch
import torch.distributions.transforms as TT

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
    return _u(x) if isinstance(x, Tensor) else torch.as_tensor(x)


class Transform:
    _type = Type.BIJECTION
    _t = None

    @classmethod
    def _is_injective(cls):
        return Type.is_injective(cls._type)

    def __call__(self, x):
        from . import Distribution, TransformedDistribution
        if isinstance(x, Distribution):
            return TransformedDistribution(x, [self])
        if isinstance(x, Transform):
            return ChainTransform([x, self])
        return self.forward(x)

    def forward(self, x):
        return Tensor(self._t(_v(x)))

    def inverse(self, y):
        return Tensor(self._t.inv(_v(y)))

    def forward_log_det_jacobian(self, x):
        x = _v(x)
        return Tensor(self._t.log_abs_det_jacobian(x, self._t(x)))

    def inverse_log_det_jacobian(self, y):
        y = _v(y)
        return Tensor(-self._t.log_abs_det_jacobian(self._t.inv(y), y))

    def forward_shape(self, shape):
        return list(self._t.forward_shape(tuple(shape)))

    def inverse_shape(self, shape):
        return list(self._t.inverse_shape(tuple(shape)))

    @property
    def _domain(self):
        return self._t.domain

    @property
    def _codomain(self):
        return self._t.codomain


class AbsTransform(Transform):
    """y = |x| (surjective): inverse returns the two preimages (-y, y)."""
    _type = Type.SURJECTION

    def forward(self, x):
        return Tensor(_v(x).abs())

    def inverse(self, y):
        y = _v(y)
        return Tensor(-y), Tensor(y)

    def forward_log_det_jacobian(self, x):
        return Tensor(torch.zeros_like(_v(x)))

    def inverse_log_det_jacobian(self, y):
        z = torch.zeros_like(_v(y))
        return Tensor(z), Tensor(z)

    def forward_shape(self, shape):
        return list(shape)

    def inverse_shape(self, shape):
        return list(shape)


class AffineTransform(Transform):
    def __init__(self, loc, scale):
        self.loc, self.scale = loc, scale
        self._t = TT.AffineTransform(_v(loc), _v(scale))


class ExpTransform(Transform):
    def __init__(self):
        self._t = TT.ExpTransform()


class PowerTransform(Transform):
    def __init__(self, power):
        self.power = power
        self._t = TT.PowerTransform(_v(power))


class SigmoidTransform(Transform):
    def __init__(self):
        self._t = TT.SigmoidTransform()


class TanhTransform(Transform):
    def __init__(self):
        self._t = TT.TanhTransform()


class SoftmaxTransform(Transform):
    _type = Type.OTHER

    def __init__(self):
        self._t = TT.SoftmaxTransform()

    def forward_log_det_jacobian(self, x):
        raise NotImplementedError("SoftmaxTransform is not injective")


class StickBreakingTransform(Transform):
    def __init__(self):
        self._t = TT.StickBreakingTransform()


class ReshapeTransform(Transform):
    def __init__(self, in_event_shape, out_event_shape):
        if math.prod(in_event_shape) != math.prod(out_event_shape):
            raise ValueError("in_event_shape and out_event_shape must have the same size")
        self.in_event_shape, self.out_event_shape = tuple(in_event_shape), tuple(out_event_shape)
        self._t = TT.ReshapeTransform(torch.Size(in_event_shape), torch.Size(out_event_shape))


class ChainTransform(Transform):
    def __init__(self, transforms):
        self.transforms = list(transforms)
        self._t = TT.ComposeTransform([t._t for t in self.transforms])

    @property
    def _type(self):
        return Type.BIJECTION if all(t._is_injective() for t in self.transforms) else Type.OTHER


class IndependentTransform(Transform):
    def __init__(self, base, reinterpreted_batch_rank):
        self.base, self.reinterpreted_batch_rank = base, reinterpreted_batch_rank
        self._t = TT.IndependentTransform(base._t, reinterpreted_batch_rank)


class StackTransform(Transform):
    def __init__(self, transforms, axis=0):
        self.transforms, self.axis = list(transforms), axis
        self._t = TT.StackTransform([t._t for t in self.transforms], axis)
