"""paddle.distribution (parity: python/paddle/distribution/__init__.py): probability
distributions with densities, moments, entropies and (reparameterised) samplers written as
tensor math, bijective transforms, and a class-pair KL registry."""
from .distribution import Distribution, ExponentialFamily, Independent, TransformedDistribution  # noqa: F401
from .continuous import Beta, Dirichlet, Gumbel, Laplace, LogNormal, Normal, Uniform  # noqa: F401
from .discrete import Categorical, Multinomial  # noqa: F401
from .kl import kl_divergence, register_kl  # noqa: F401
from . import transform  # noqa: F401
from .transform import *  # noqa: F401,F403

__all__ = ['Beta', 'Categorical', 'Dirichlet', 'Distribution', 'ExponentialFamily', 'Multinomial',
           'Normal', 'Uniform', 'kl_divergence', 'register_kl', 'Independent', 'TransformedDistribution',
           'Laplace', 'LogNormal', 'Gumbel'] + list(transform.__all__)
