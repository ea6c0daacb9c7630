"""paddle.framework (parity: python/paddle/framework/__init__.py)."""
from .core import (Tensor, Parameter, EagerParamBase, Place, CPUPlace, CUDAPlace,  # noqa
                   in_dynamic_mode, set_default_dtype, get_default_dtype, no_grad, convert_dtype)
from .core import in_dygraph_mode  # noqa
from .io import save, load  # noqa
from .flags import set_flags, get_flags  # noqa
from ..tensor.random import seed, get_rng_state, set_rng_state  # noqa


def core():
    return None
