"""Distribution base classes (parity: python/paddle/distribution/distribution.py,
exponential_family.py, independent.py, transformed_distribution.py).

Every density / sampler in this package is written out here as tensor math on the framework's
tensors (no torch.distributions objects): sampling draws from the framework generator
(``paddle.seed``), reparameterised samplers keep gradients to the parameters, and everything runs
on the parameters' device.
"""
import math

import torch

from ..framework.core import Tensor, _u

__all__ = ['Distribution', 'ExponentialFamily', 'Independent', 'TransformedDistribution']


def _param(x, dtype=None):
    """A parameter as a float tensor (python numbers / numpy / paddle Tensors)."""
    if isinstance(x, Tensor):
        t = x._t
    elif isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.as_tensor(x)
    if not t.is_floating_point():
        t = t.to(dtype or torch.get_default_dtype())
    elif dtype is not None:
        t = t.to(dtype)
    return t


def _value(x, like=None):
    t = _u(x) if isinstance(x, Tensor) else torch.as_tensor(x)
    if like is not None:
        if t.is_floating_point() and like.is_floating_point():
            t = t.to(like.dtype)
        t = t.to(like.device)
    return t


def _extend(shape, batch_shape, event_shape=()):
    return tuple(shape) + tuple(batch_shape) + tuple(event_shape)


class Distribution:
    """Abstract distribution with ``batch_shape`` (independent, non-identical copies) and
    ``event_shape`` (the shape of one draw)."""

    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return list(self._batch_shape)

    @property
    def event_shape(self):
        return list(self._event_shape)

    @property
    def mean(self):
        raise NotImplementedError

    @property
    def variance(self):
        raise NotImplementedError

    @property
    def stddev(self):
        return Tensor(_u(self.variance).sqrt())

    def _extend_shape(self, sample_shape):
        return _extend(sample_shape, self._batch_shape, self._event_shape)

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return Tensor(self._rsample(tuple(shape)).detach())

    def rsample(self, shape=()):
        return Tensor(self._rsample(tuple(shape)))

    def _rsample(self, shape):
        raise NotImplementedError(f"{type(self).__name__} has no reparameterised sampler")

    def log_prob(self, value):
        return Tensor(self._log_prob(_value(value, self._ref())))

    def prob(self, value):
        return Tensor(self._log_prob(_value(value, self._ref())).exp())

    probs = prob

    def entropy(self):
        return Tensor(self._entropy())

    def kl_divergence(self, other):
        from .kl import kl_divergence
        return kl_divergence(self, other)

    # helpers
    def _ref(self):
        raise NotImplementedError

    def _log_prob(self, v):
        raise NotImplementedError

    def _entropy(self):
        raise NotImplementedError

    def __repr__(self):
        return f"{type(self).__name__}(batch_shape={self.batch_shape}, event_shape={self.event_shape})"


class ExponentialFamily(Distribution):
    """p(x) = h(x) exp(<eta, T(x)> - A(eta)). The entropy follows from the log-normaliser A:
    H = A(eta) - <eta, grad A(eta)> - E[log h(x)], with grad A by autograd; subclasses provide
    ``_natural_parameters``, ``_log_normalizer`` and ``_mean_carrier_measure``."""

    @property
    def _natural_parameters(self):
        raise NotImplementedError

    def _log_normalizer(self, *natural):
        raise NotImplementedError

    @property
    def _mean_carrier_measure(self):
        raise NotImplementedError

    def _entropy(self):
        eta = [p.detach().requires_grad_(True) for p in self._natural_parameters]
        with torch.enable_grad():
            a = self._log_normalizer(*eta)
            grads = torch.autograd.grad(a.sum(), eta, create_graph=True)
        h = a - self._mean_carrier_measure
        for e, g in zip(eta, grads):
            h = h - (e * g).reshape(a.shape + (-1,)).sum(-1)
        return h if any(p.requires_grad for p in self._natural_parameters) else h.detach()


class Independent(Distribution):
    """Reinterprets the rightmost ``reinterpreted_batch_rank`` batch dims of ``base`` as event
    dims: log_prob / entropy sum over them."""

    def __init__(self, base, reinterpreted_batch_rank):
        if not 0 < reinterpreted_batch_rank <= len(base.batch_shape):
            raise ValueError(f"reinterpreted_batch_rank must be in (0, {len(base.batch_shape)}], "
                             f"got {reinterpreted_batch_rank}")
        self.base, self.reinterpreted_batch_rank = base, reinterpreted_batch_rank
        bs = base.batch_shape
        k = len(bs) - reinterpreted_batch_rank
        super().__init__(bs[:k], bs[k:] + base.event_shape)

    def _sum_right(self, t):
        return t.sum(tuple(range(-self.reinterpreted_batch_rank, 0))) if self.reinterpreted_batch_rank else t

    @property
    def mean(self):
        return self.base.mean

    @property
    def variance(self):
        return self.base.variance

    def _ref(self):
        return self.base._ref()

    def _rsample(self, shape):
        return self.base._rsample(shape)

    def sample(self, shape=(), seed=0):
        return self.base.sample(shape)

    def _log_prob(self, v):
        return self._sum_right(self.base._log_prob(v))

    def _entropy(self):
        return self._sum_right(self.base._entropy())


def _sum_to_ndim(t, nd):
    """Sum the trailing dims of ``t`` until it has ``nd`` dims."""
    if not isinstance(t, torch.Tensor):
        return t
    extra = t.dim() - nd
    return t.sum(tuple(range(-extra, 0))) if extra > 0 else t


class TransformedDistribution(Distribution):
    """y = T(x), x ~ base, T = T_n o ... o T_1: log p(y) = log p_base(T^-1 y) - log|det J_T(x)|
    (change of variables), with both terms summed over the event dims of y."""

    def __init__(self, base, transforms):
        from .transform import ChainTransform, Transform
        if not isinstance(base, Distribution):
            raise TypeError("base must be a Distribution")
        transforms = list(transforms)
        if not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("transforms must be Transform instances")
        self.base, self.transforms = base, transforms
        self._chain = ChainTransform(transforms)
        shape = self._chain.forward_shape(base.batch_shape + base.event_shape)
        ev_in = max(len(base.event_shape), self._chain._event_rank_in)
        ev_out = ev_in + self._chain._event_rank - self._chain._event_rank_in
        cut = len(shape) - ev_out
        super().__init__(shape[:cut], shape[cut:])

    def _ref(self):
        return self.base._ref()

    def _rsample(self, shape):
        return self._chain._fwd(self.base._rsample(shape))

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return Tensor(self._chain._fwd(_u(self.base.sample(shape))))

    def _log_prob(self, y):
        x = self._chain._inv(y)
        nd = y.dim() - len(self._event_shape)
        return _sum_to_ndim(self.base._log_prob(x), nd) - _sum_to_ndim(self._chain._fldj(x), nd)


_LOG_SQRT_2PI = 0.5 * math.log(2 * math.pi)
