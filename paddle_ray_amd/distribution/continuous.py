"""Continuous distributions (parity: python/paddle/distribution/{normal,uniform,beta,dirichlet,
laplace,lognormal,gumbel}.py): densities, moments, entropies and samplers as tensor math."""
import math

import torch

from ..framework.core import Tensor, _u
from .distribution import (Distribution, ExponentialFamily, TransformedDistribution, _LOG_SQRT_2PI,
                           _param)
from .transform import ExpTransform

__all__ = ['Normal', 'Uniform', 'Beta', 'Dirichlet', 'Laplace', 'LogNormal', 'Gumbel']

_EULER = 0.5772156649015329


def _bcast(*ts):
    ts = [_param(t) for t in ts]
    dt = torch.promote_types(*[t.dtype for t in ts]) if len(ts) > 1 else ts[0].dtype
    dev = next((t.device for t in ts if t.device.type != 'cpu'), ts[0].device)
    return torch.broadcast_tensors(*[t.to(dtype=dt, device=dev) for t in ts])


class Normal(ExponentialFamily):
    """N(loc, scale^2)."""

    def __init__(self, loc, scale, name=None):
        self.loc, self.scale = _bcast(loc, scale)
        super().__init__(self.loc.shape)

    def _ref(self):
        return self.loc

    @property
    def mean(self):
        return Tensor(self.loc)

    @property
    def variance(self):
        return Tensor(self.scale ** 2)

    @property
    def stddev(self):
        return Tensor(self.scale)

    def _rsample(self, shape):
        eps = torch.randn(self._extend_shape(shape), dtype=self.loc.dtype, device=self.loc.device)
        return self.loc + self.scale * eps

    def _log_prob(self, v):
        z = (v - self.loc) / self.scale
        return -0.5 * z * z - self.scale.log() - _LOG_SQRT_2PI

    def _entropy(self):
        return 0.5 + _LOG_SQRT_2PI + self.scale.log()

    def cdf(self, value):
        v = _param(value).to(self.loc)
        return Tensor(0.5 * (1 + torch.erf((v - self.loc) / (self.scale * math.sqrt(2)))))

    def icdf(self, value):
        v = _param(value).to(self.loc)
        return Tensor(self.loc + self.scale * torch.erfinv(2 * v - 1) * math.sqrt(2))

    @property
    def _natural_parameters(self):
        return (self.loc / self.scale ** 2, -0.5 / self.scale ** 2)

    def _log_normalizer(self, x, y):
        return -0.25 * x * x / y + 0.5 * torch.log(-math.pi / y)

    @property
    def _mean_carrier_measure(self):
        return 0.0


class Uniform(Distribution):
    """U[low, high)."""

    def __init__(self, low, high, name=None):
        self.low, self.high = _bcast(low, high)
        super().__init__(self.low.shape)

    def _ref(self):
        return self.low

    @property
    def mean(self):
        return Tensor((self.low + self.high) / 2)

    @property
    def variance(self):
        return Tensor((self.high - self.low) ** 2 / 12)

    def _rsample(self, shape):
        u = torch.rand(self._extend_shape(shape), dtype=self.low.dtype, device=self.low.device)
        return self.low + (self.high - self.low) * u

    def _log_prob(self, v):
        inside = (v >= self.low) & (v < self.high)
        lp = -(self.high - self.low).log()
        return torch.where(inside, lp, torch.full_like(lp, -math.inf))

    def _entropy(self):
        return (self.high - self.low).log()

    def cdf(self, value):
        v = _param(value).to(self.low)
        return Tensor(((v - self.low) / (self.high - self.low)).clamp(0, 1))


def _sample_gamma(alpha):
    """Gamma(alpha, 1) draws with gradients w.r.t. alpha (implicit reparameterisation)."""
    return torch._standard_gamma(alpha)


class Dirichlet(ExponentialFamily):
    """Dir(concentration) on the simplex of the last dim."""

    def __init__(self, concentration, name=None):
        c = _param(concentration)
        if c.dim() < 1:
            raise ValueError("concentration must have at least one dimension")
        self.concentration = c
        super().__init__(c.shape[:-1], c.shape[-1:])

    def _ref(self):
        return self.concentration

    @property
    def mean(self):
        c = self.concentration
        return Tensor(c / c.sum(-1, keepdim=True))

    @property
    def variance(self):
        c = self.concentration
        c0 = c.sum(-1, keepdim=True)
        return Tensor(c * (c0 - c) / (c0 ** 2 * (c0 + 1)))

    def _rsample(self, shape):
        c = self.concentration.expand(self._extend_shape(shape))
        g = _sample_gamma(c)
        return g / g.sum(-1, keepdim=True)

    def _log_prob(self, v):
        c = self.concentration
        return (torch.xlogy(c - 1, v).sum(-1) + torch.lgamma(c.sum(-1)) - torch.lgamma(c).sum(-1))

    def _entropy(self):
        c = self.concentration
        k = c.shape[-1]
        c0 = c.sum(-1)
        lnb = torch.lgamma(c).sum(-1) - torch.lgamma(c0)
        return lnb + (c0 - k) * torch.digamma(c0) - ((c - 1) * torch.digamma(c)).sum(-1)

    @property
    def _natural_parameters(self):
        return (self.concentration,)

    def _log_normalizer(self, x):
        return torch.lgamma(x).sum(-1) - torch.lgamma(x.sum(-1))


class Beta(ExponentialFamily):
    """Beta(alpha, beta) = the first coordinate of Dir([alpha, beta])."""

    def __init__(self, alpha, beta, name=None):
        self.alpha, self.beta = _bcast(alpha, beta)
        super().__init__(self.alpha.shape)

    def _ref(self):
        return self.alpha

    @property
    def mean(self):
        return Tensor(self.alpha / (self.alpha + self.beta))

    @property
    def variance(self):
        s = self.alpha + self.beta
        return Tensor(self.alpha * self.beta / (s ** 2 * (s + 1)))

    def _rsample(self, shape):
        a = self.alpha.expand(self._extend_shape(shape))
        b = self.beta.expand(self._extend_shape(shape))
        ga, gb = _sample_gamma(a), _sample_gamma(b)
        return ga / (ga + gb)

    def _log_prob(self, v):
        a, b = self.alpha, self.beta
        return (torch.xlogy(a - 1, v) + torch.xlogy(b - 1, 1 - v) + torch.lgamma(a + b) - torch.lgamma(a)
                - torch.lgamma(b))

    def _entropy(self):
        a, b = self.alpha, self.beta
        s = a + b
        lnb = torch.lgamma(a) + torch.lgamma(b) - torch.lgamma(s)
        return lnb - (a - 1) * torch.digamma(a) - (b - 1) * torch.digamma(b) + (s - 2) * torch.digamma(s)

    @property
    def _natural_parameters(self):
        return (self.alpha, self.beta)

    def _log_normalizer(self, x, y):
        return torch.lgamma(x) + torch.lgamma(y) - torch.lgamma(x + y)


class Laplace(Distribution):
    """Laplace(loc, scale): density exp(-|x - loc| / scale) / (2 scale)."""

    def __init__(self, loc, scale, name=None):
        self.loc, self.scale = _bcast(loc, scale)
        if bool((self.scale <= 0).any()):
            raise ValueError("Laplace scale must be positive")
        super().__init__(self.loc.shape)

    def _ref(self):
        return self.loc

    @property
    def mean(self):
        return Tensor(self.loc)

    @property
    def variance(self):
        return Tensor(2 * self.scale ** 2)

    @property
    def stddev(self):
        return Tensor(math.sqrt(2) * self.scale)

    def _rsample(self, shape):
        eps = torch.finfo(self.loc.dtype).eps
        u = torch.rand(self._extend_shape(shape), dtype=self.loc.dtype, device=self.loc.device)
        u = (2 * u - 1).clamp(-1 + eps, 1 - eps)
        return self.loc - self.scale * u.sign() * torch.log1p(-u.abs())

    def _log_prob(self, v):
        return -(v - self.loc).abs() / self.scale - torch.log(2 * self.scale)

    def _entropy(self):
        return 1 + torch.log(2 * self.scale)

    def cdf(self, value):
        v = _param(value).to(self.loc)
        z = (v - self.loc) / self.scale
        return Tensor(0.5 - 0.5 * z.sign() * torch.expm1(-z.abs()))

    def icdf(self, value):
        p = _param(value).to(self.loc)
        t = p - 0.5
        return Tensor(self.loc - self.scale * t.sign() * torch.log1p(-2 * t.abs()))


class LogNormal(TransformedDistribution):
    """exp(X), X ~ N(loc, scale^2)."""

    def __init__(self, loc, scale, name=None):
        self._base = Normal(loc, scale)
        self.loc, self.scale = self._base.loc, self._base.scale
        super().__init__(self._base, [ExpTransform()])

    @property
    def mean(self):
        return Tensor(torch.exp(self.loc + self.scale ** 2 / 2))

    @property
    def variance(self):
        s2 = self.scale ** 2
        return Tensor(torch.expm1(s2) * torch.exp(2 * self.loc + s2))

    def _entropy(self):
        return self._base._entropy() + self.loc


class Gumbel(TransformedDistribution):
    """Gumbel(loc, scale): loc - scale * log(-log U)."""

    def __init__(self, loc, scale, name=None):
        self.loc, self.scale = _bcast(loc, scale)
        from .transform import AffineTransform
        base = Uniform(torch.zeros_like(self.loc), torch.ones_like(self.loc))
        self._aff = AffineTransform(self.loc, self.scale)
        Distribution.__init__(self, self.loc.shape)
        self.base, self.transforms = base, [self._aff]

    def _ref(self):
        return self.loc

    @property
    def mean(self):
        return Tensor(self.loc + self.scale * _EULER)

    @property
    def variance(self):
        return Tensor(math.pi ** 2 / 6 * self.scale ** 2)

    @property
    def stddev(self):
        return Tensor(math.pi / math.sqrt(6) * self.scale)

    def _rsample(self, shape):
        tiny = torch.finfo(self.loc.dtype).tiny
        u = torch.rand(self._extend_shape(shape), dtype=self.loc.dtype, device=self.loc.device)
        u = u.clamp(tiny, 1 - torch.finfo(self.loc.dtype).eps)
        return self.loc - self.scale * torch.log(-torch.log(u))

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return Tensor(self._rsample(tuple(shape)))

    def _log_prob(self, v):
        z = (v - self.loc) / self.scale
        return -(z + torch.exp(-z)) - self.scale.log()

    def _entropy(self):
        return self.scale.log() + 1 + _EULER

    def cdf(self, value):
        v = _param(value).to(self.loc)
        return Tensor(torch.exp(-torch.exp(-(v - self.loc) / self.scale)))
