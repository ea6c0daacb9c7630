"""Discrete distributions (parity: python/paddle/distribution/{categorical,multinomial}.py)."""
import torch

from ..framework.core import Tensor, _u
from .distribution import Distribution, _param

__all__ = ['Categorical', 'Multinomial']


class Categorical(Distribution):
    """Categorical over the last dim of ``logits`` (unnormalised log-probabilities; the
    reference accepts non-negative weights too: both are normalised the same way here, by
    ``logits - logsumexp``)."""

    def __init__(self, logits, name=None):
        lg = _param(logits)
        self.logits = lg - torch.logsumexp(lg, -1, keepdim=True)
        super().__init__(lg.shape[:-1])

    def _ref(self):
        return self.logits

    @property
    def _probs(self):
        return self.logits.exp()

    @property
    def mean(self):
        raise NotImplementedError("Categorical has no mean")

    def sample(self, shape=(), seed=0):
        shape = tuple(shape)
        p = self._probs.reshape(-1, self.logits.shape[-1])
        n = 1
        for s in shape:
            n *= s
        idx = torch.multinomial(p, max(n, 1), replacement=True)  # [batch, n]
        idx = idx.t().reshape(shape + self._batch_shape)
        return Tensor(idx.to(torch.int64))

    def _gather(self, t, value):
        v = value.to(t.device).long()
        shp = torch.broadcast_shapes(v.shape, t.shape[:-1])
        return t.expand(*shp, t.shape[-1]).gather(-1, v.expand(shp).unsqueeze(-1)).squeeze(-1)

    def _log_prob(self, value):
        return self._gather(self.logits, value)

    def log_prob(self, value):
        return Tensor(self._log_prob(_u(value) if hasattr(value, '_t') else torch.as_tensor(value)))

    def probs(self, value):
        """Probability of each category in ``value`` (reference name)."""
        return Tensor(self._gather(self._probs, _u(value) if hasattr(value, '_t') else torch.as_tensor(value)))

    prob = probs

    def _entropy(self):
        p = self._probs
        return -(p * self.logits).sum(-1)

    def kl_divergence(self, other):
        p = self._probs
        return Tensor((p * (self.logits - other.logits)).sum(-1))


class Multinomial(Distribution):
    """Counts of ``total_count`` draws from the categories of ``probs``."""

    def __init__(self, total_count, probs, name=None):
        if int(total_count) < 1:
            raise ValueError("total_count must be >= 1")
        p = _param(probs)
        self.total_count = int(total_count)
        self.probs_ = p / p.sum(-1, keepdim=True)
        super().__init__(p.shape[:-1], p.shape[-1:])

    @property
    def probs(self):
        return Tensor(self.probs_)

    def _ref(self):
        return self.probs_

    @property
    def mean(self):
        return Tensor(self.total_count * self.probs_)

    @property
    def variance(self):
        return Tensor(self.total_count * self.probs_ * (1 - self.probs_))

    def sample(self, shape=(), seed=0):
        shape = tuple(shape)
        k = self.probs_.shape[-1]
        p = self.probs_.reshape(-1, k)
        n = 1
        for s in shape:
            n *= s
        draws = torch.multinomial(p, self.total_count * max(n, 1), replacement=True)
        draws = draws.view(p.shape[0], max(n, 1), self.total_count)
        counts = torch.zeros(p.shape[0], max(n, 1), k, dtype=p.dtype, device=p.device)
        counts.scatter_add_(-1, draws, torch.ones_like(draws, dtype=p.dtype))
        counts = counts.permute(1, 0, 2).reshape(shape + self._batch_shape + (k,))
        return Tensor(counts)

    def _log_prob(self, v):
        v = v.to(self.probs_.dtype)
        logp = torch.xlogy(v, self.probs_).sum(-1)
        return logp + torch.lgamma(v.sum(-1) + 1) - torch.lgamma(v + 1).sum(-1)

    def _entropy(self):
        # H = -sum_x p(x) log p(x) over the support (counts summing to n): exact for the small
        # supports the reference evaluates, via lgamma / binomial marginals:
        # H = -lgamma(n+1) - n sum p_i log p_i + sum_i sum_{k=0..n} Binom(k; n, p_i) lgamma(k+1)
        n = self.total_count
        p = self.probs_
        k = torch.arange(n + 1, dtype=p.dtype, device=p.device)
        logc = torch.lgamma(torch.tensor(n + 1.0, dtype=p.dtype)) - torch.lgamma(k + 1) - \
            torch.lgamma(n - k + 1)
        pk = p.unsqueeze(-1)
        binom = torch.exp(logc + torch.xlogy(k, pk) + torch.xlogy(n - k, 1 - pk))
        return (-torch.lgamma(torch.tensor(n + 1.0, dtype=p.dtype)) - n * torch.xlogy(p, p).sum(-1)
                + (binom * torch.lgamma(k + 1)).sum((-1, -2)))
