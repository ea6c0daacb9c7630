"""paddle.static (parity: python/paddle/static/__init__.py)."""
_STATIC = [False]


def _static_mode_enabled():
    return _STATIC[0]


from .program import *  # noqa: E402,F401,F403
from .input import InputSpec  # noqa: E402,F401
