"""KL divergences (parity: python/paddle/distribution/kl.py): a registry keyed by the two
distribution classes, resolved to the most specific registered pair (MRO distance), with the
closed forms of the pairs below."""
import math

import torch

from ..framework.core import Tensor
from .continuous import Beta, Dirichlet, Gumbel, Laplace, LogNormal, Normal, Uniform
from .discrete import Categorical, Multinomial
from .distribution import Distribution, ExponentialFamily, Independent

__all__ = ['kl_divergence', 'register_kl']

_REGISTRY = {}


def register_kl(cls_p, cls_q):
    """Decorator: ``fn(p, q)`` computes KL(p || q) for instances of the two classes."""
    if not (issubclass(cls_p, Distribution) and issubclass(cls_q, Distribution)):
        raise TypeError("register_kl takes two Distribution subclasses")

    def deco(fn):
        _REGISTRY[(cls_p, cls_q)] = fn
        return fn
    return deco


def _dispatch(cp, cq):
    best, score = None, None
    for (a, b), fn in _REGISTRY.items():
        if issubclass(cp, a) and issubclass(cq, b):
            s = (cp.__mro__.index(a), cq.__mro__.index(b))
            if score is None or s < score:
                best, score = fn, s
    return best


def kl_divergence(p, q):
    """KL(p || q) = E_p[log p - log q]."""
    fn = _dispatch(type(p), type(q))
    if fn is None:
        raise NotImplementedError(f"no KL divergence registered for {type(p).__name__} || {type(q).__name__}")
    r = fn(p, q)
    return r if isinstance(r, Tensor) else Tensor(r)


@register_kl(Normal, Normal)
def _kl_normal(p, q):
    vr = (p.scale / q.scale) ** 2
    t = ((p.loc - q.loc) / q.scale) ** 2
    return 0.5 * (vr + t - 1 - vr.log())


@register_kl(Uniform, Uniform)
def _kl_uniform(p, q):
    r = ((q.high - q.low) / (p.high - p.low)).log()
    outside = (q.low > p.low) | (q.high < p.high)
    return torch.where(outside, torch.full_like(r, math.inf), r)


@register_kl(Beta, Beta)
def _kl_beta(p, q):
    a1, b1, a2, b2 = p.alpha, p.beta, q.alpha, q.beta
    s1 = a1 + b1
    lnb1 = torch.lgamma(a1) + torch.lgamma(b1) - torch.lgamma(s1)
    lnb2 = torch.lgamma(a2) + torch.lgamma(b2) - torch.lgamma(a2 + b2)
    return (lnb2 - lnb1 + (a1 - a2) * torch.digamma(a1) + (b1 - b2) * torch.digamma(b1)
            + (a2 - a1 + b2 - b1) * torch.digamma(s1))


@register_kl(Dirichlet, Dirichlet)
def _kl_dirichlet(p, q):
    c1, c2 = p.concentration, q.concentration
    s1 = c1.sum(-1)
    return (torch.lgamma(s1) - torch.lgamma(c2.sum(-1)) - (torch.lgamma(c1) - torch.lgamma(c2)).sum(-1)
            + ((c1 - c2) * (torch.digamma(c1) - torch.digamma(s1).unsqueeze(-1))).sum(-1))


@register_kl(Categorical, Categorical)
def _kl_categorical(p, q):
    return (p._probs * (p.logits - q.logits)).sum(-1)


@register_kl(Laplace, Laplace)
def _kl_laplace(p, q):
    d = (p.loc - q.loc).abs()
    r = p.scale / q.scale
    return -r.log() + d / q.scale + r * torch.exp(-d / p.scale) - 1


@register_kl(LogNormal, LogNormal)
def _kl_lognormal(p, q):
    return _kl_normal(p._base, q._base)


@register_kl(Gumbel, Gumbel)
def _kl_gumbel(p, q):
    ct1, ct2 = p.scale / q.scale, q.loc / q.scale
    ct3 = p.loc / q.scale
    t1 = -ct1.log() - ct2 + ct3
    t2 = ct1 * 0.5772156649015329
    t3 = torch.exp(ct2 + torch.lgamma(1 + ct1) - ct3)
    return t1 + t2 + t3 - (1 + 0.5772156649015329)


@register_kl(Independent, Independent)
def _kl_independent(p, q):
    if p.reinterpreted_batch_rank != q.reinterpreted_batch_rank:
        raise NotImplementedError("Independent KL needs equal reinterpreted_batch_rank")
    from .kl import kl_divergence as _k
    r = _k(p.base, q.base)._t
    return r.sum(tuple(range(-p.reinterpreted_batch_rank, 0)))


@register_kl(ExponentialFamily, ExponentialFamily)
def _kl_expfamily(p, q):
    """Same-family Bregman divergence of the log-normaliser:
    KL = A(eta_q) - A(eta_p) - <eta_q - eta_p, grad A(eta_p)>."""
    if type(p) is not type(q):
        raise NotImplementedError(f"no KL divergence for {type(p).__name__} || {type(q).__name__}")
    ep = [t.detach().requires_grad_(True) for t in p._natural_parameters]
    eq = list(q._natural_parameters)
    with torch.enable_grad():
        ap = p._log_normalizer(*ep)
        grads = torch.autograd.grad(ap.sum(), ep, create_graph=True)
    r = q._log_normalizer(*eq) - ap
    for a, b, g in zip(eq, ep, grads):
        r = r - ((a - b) * g).reshape(ap.shape + (-1,)).sum(-1)
    need = any(t.requires_grad for t in list(p._natural_parameters) + eq)
    return r if need else r.detach()
