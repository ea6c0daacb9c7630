"""Random API + RNG state (parity: python/paddle/tensor/random.py, python/paddle/framework/random.py).

One generator per device (torch's Philox on the HIP device); ``get_rng_state``
returns per-device states so recompute / TP RNG trackers can fork and restore.
"""
import numpy as np
import torch

from ..framework.core import Tensor, _u, convert_dtype, get_default_dtype, _default_device
from .creation import _shape


def _dt(d):
    return convert_dtype(d) or get_default_dtype()


def seed(s):
    s = int(s)
    torch.manual_seed(s)
    np.random.seed(s % (2 ** 32))
    return torch.default_generator


def get_rng_state(device=None):
    states = [torch.get_rng_state()]
    if torch.cuda.is_available():
        states += list(torch.cuda.get_rng_state_all())
    return states


def set_rng_state(state_list, device=None):
    torch.set_rng_state(state_list[0])
    if torch.cuda.is_available() and len(state_list) > 1:
        torch.cuda.set_rng_state_all(state_list[1:])


def get_cuda_rng_state():
    return list(torch.cuda.get_rng_state_all()) if torch.cuda.is_available() else []


def set_cuda_rng_state(state_list):
    if torch.cuda.is_available() and state_list:
        torch.cuda.set_rng_state_all(state_list)


def rand(shape, dtype=None, name=None):
    return Tensor(torch.rand(_shape(shape), dtype=_dt(dtype), device=_default_device()))


def randn(shape, dtype=None, name=None):
    return Tensor(torch.randn(_shape(shape), dtype=_dt(dtype), device=_default_device()))


standard_normal = randn


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):
    t = torch.empty(_shape(shape), dtype=_dt(dtype), device=_default_device())
    g = None
    if seed:
        g = torch.Generator(device=t.device).manual_seed(seed)
    return Tensor(t.uniform_(min, max, generator=g))


def uniform_(x, min=-1.0, max=1.0, seed=0, name=None):
    with torch.no_grad():
        x._t.uniform_(min, max)
    return x


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if isinstance(mean, Tensor) or isinstance(std, Tensor):
        m = _u(mean) if isinstance(mean, Tensor) else torch.tensor(mean)
        s = _u(std) if isinstance(std, Tensor) else torch.tensor(std)
        return Tensor(torch.normal(m, s))
    return Tensor(torch.normal(float(mean), float(std), _shape(shape), dtype=get_default_dtype(),
                               device=_default_device()))


def normal_(x, mean=0.0, std=1.0, name=None):
    with torch.no_grad():
        x._t.normal_(mean, std)
    return x


def gaussian(shape, mean=0.0, std=1.0, seed=0, dtype=None, name=None):
    return Tensor(torch.normal(float(mean), float(std), _shape(shape), dtype=_dt(dtype),
                               device=_default_device()))


def randint(low=0, high=None, shape=[1], dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return Tensor(torch.randint(low, high, _shape(shape), dtype=convert_dtype(dtype) or torch.int64,
                                device=_default_device()))


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    t = _u(x)
    return Tensor(torch.randint(low, high, t.shape, dtype=convert_dtype(dtype) or t.dtype,
                                device=t.device))


def randperm(n, dtype='int64', name=None):
    return Tensor(torch.randperm(n, dtype=convert_dtype(dtype), device=_default_device()))


def bernoulli(x, name=None):
    return Tensor(torch.bernoulli(_u(x)))


def poisson(x, name=None):
    return Tensor(torch.poisson(_u(x)))


def multinomial(x, num_samples=1, replacement=False, name=None):
    return Tensor(torch.multinomial(_u(x), num_samples, replacement))


def exponential_(x, lam=1.0, name=None):
    with torch.no_grad():
        x._t.exponential_(lam)
    return x
