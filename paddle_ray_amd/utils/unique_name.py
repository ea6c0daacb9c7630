import collections
import contextlib

import importlib

_core = importlib.import_module('paddle_ray_amd.framework.core')


def generate(key):
    return _core._unique_name(key)


@contextlib.contextmanager
def guard(new_generator=None):
    """Fresh name counters for layers / parameters / tensors created inside (parity:
    python/paddle/utils/unique_name.py guard)."""
    old = _core._NAME_COUNTERS[0]
    _core._NAME_COUNTERS[0] = collections.defaultdict(int)
    try:
        yield
    finally:
        _core._NAME_COUNTERS[0] = old
