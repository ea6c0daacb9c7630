"""paddle.utils (parity: python/paddle/utils/__init__.py)."""
import functools
import importlib
import warnings


def deprecated(update_to="", since="", reason="", level=0):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **k):
            warnings.warn(f"{fn.__name__} is deprecated since {since}: {reason}", DeprecationWarning)
            return fn(*a, **k)
        return wrapper
    return deco


def try_import(module_name, err_msg=None):
    try:
        return importlib.import_module(module_name)
    except ImportError:
        raise ImportError(err_msg or f"{module_name} is required")


def require_version(min_version, max_version=None):
    return True


def run_check():
    """paddle.utils.run_check: a tiny forward/backward on every visible device."""
    import torch
    import paddle_ray_amd as paddle
    devs = ['cpu'] + (['gpu:0'] if torch.cuda.is_available() else [])
    for d in devs:
        prev = paddle.get_device()
        paddle.set_device(d)
        lin = paddle.nn.Linear(4, 4)
        x = paddle.randn([2, 4])
        lin(x).sum().backward()
        paddle.set_device(prev)
    print(f"paddle_ray_amd is installed successfully! devices checked: {devs}")


from . import unique_name  # noqa
from .layers_utils import (flatten, pack_sequence_as, map_structure,  # noqa
                           assert_same_structure, is_sequence)
from .dlpack import to_dlpack, from_dlpack  # noqa
