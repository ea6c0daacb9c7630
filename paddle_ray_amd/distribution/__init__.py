"""paddle.distribution (parity: python/paddle/distribution/*) over torch.distributions."""
import torch
import torch.distributions as D

from ..framework.core import Tensor, _u


def _t(x):
    if isinstance(x, Tensor):
        return x._t
    return torch.as_tensor(x, dtype=torch.float32)


class Distribution:
    _d = None

    @property
    def batch_shape(self):
        return list(self._d.batch_shape)

    @property
    def event_shape(self):
        return list(self._d.event_shape)

    @property
    def mean(self):
        return Tensor(self._d.mean)

    @property
    def variance(self):
        return Tensor(self._d.variance)

    def sample(self, shape=()):
        return Tensor(self._d.sample(tuple(shape)))

    def rsample(self, shape=()):
        return Tensor(self._d.rsample(tuple(shape)))

    def log_prob(self, value):
        return Tensor(self._d.log_prob(_t(value)))

    def prob(self, value):
        return Tensor(self._d.log_prob(_t(value)).exp())

    def entropy(self):
        return Tensor(self._d.entropy())

    def kl_divergence(self, other):
        return Tensor(D.kl_divergence(self._d, other._d))


class ExponentialFamily(Distribution):
    pass


def _mk(name, ctor):
    def __init__(self, *args, **kw):
        self._d = ctor(*[_t(a) for a in args], **{k: _t(v) for k, v in kw.items()
                                                  if k != 'name'})
    return type(name, (ExponentialFamily,), {'__init__': __init__})


Normal = _mk('Normal', D.Normal)
Uniform = _mk('Uniform', D.Uniform)
Beta = _mk('Beta', D.Beta)
Dirichlet = _mk('Dirichlet', D.Dirichlet)
Laplace = _mk('Laplace', D.Laplace)
LogNormal = _mk('LogNormal', D.LogNormal)
Gumbel = _mk('Gumbel', D.Gumbel)


class Categorical(Distribution):
    def __init__(self, logits, name=None):
        self._d = D.Categorical(logits=_t(logits))

    def probs(self, value):
        return Tensor(self._d.probs.gather(-1, _t(value).long().unsqueeze(-1)).squeeze(-1))


class Multinomial(Distribution):
    def __init__(self, total_count, probs):
        self._d = D.Multinomial(int(total_count), probs=_t(probs))


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_rank):
        self._d = D.Independent(base._d, reinterpreted_batch_rank)


class TransformedDistribution(Distribution):
    def __init__(self, base, transforms):
        self._d = D.TransformedDistribution(base._d, [t._t for t in transforms])


_KL_REGISTRY = {}


def kl_divergence(p, q):
    """KL(p || q): user registrations (register_kl) first, then the closed forms."""
    for (cp, cq), fn in _KL_REGISTRY.items():
        if isinstance(p, cp) and isinstance(q, cq):
            return fn(p, q)
    return Tensor(D.kl_divergence(p._d, q._d))


def register_kl(cls_p, cls_q):
    """Decorator registering ``fn(p, q)`` as KL(p || q) for the two distribution classes."""
    def deco(fn):
        _KL_REGISTRY[(cls_p, cls_q)] = fn
        return fn
    return deco

from . import transform  # noqa: E402
from .transform import *  # noqa: E402,F401,F403
