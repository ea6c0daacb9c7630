"""paddle.jit: to_static (HIP-graph replay), save/load via static Programs."""
from .api import to_static, not_to_static, ignore_module, save, load, TranslatedLayer, \
    StaticFunction, set_code_level, set_verbosity, enable_to_static  # noqa
from ..static.input import InputSpec  # noqa
