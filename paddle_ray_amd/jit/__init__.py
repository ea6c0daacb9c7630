"""paddle.jit placeholder (full implementation in jit/api.py)."""
from .api import to_static, not_to_static, ignore_module, save, load, TranslatedLayer, \
    set_code_level, set_verbosity, enable_to_static  # noqa
from ..static.input import InputSpec  # noqa
