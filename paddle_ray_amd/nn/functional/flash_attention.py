"""paddle.nn.functional.flash_attention (parity: python/paddle/nn/functional/flash_attention.py):
the module path of ``flash_attention`` / ``flash_attn_unpadded`` /
``scaled_dot_product_attention``; the implementations live in ``nn.functional``. Importing
this module rebinds ``nn.functional.flash_attention`` to it (Python's submodule rule), so the
module itself is callable as the function: both spellings keep working."""
import sys
import types

from . import flash_attention as _fa_fn  # the function (before this module shadows it)
from . import flash_attn_unpadded, scaled_dot_product_attention  # noqa: F401

flash_attention = _fa_fn if not isinstance(_fa_fn, types.ModuleType) else _fa_fn.flash_attention

__all__ = ['flash_attention', 'flash_attn_unpadded', 'scaled_dot_product_attention']


class _CallableModule(types.ModuleType):
    def __call__(self, *args, **kwargs):
        return flash_attention(*args, **kwargs)


sys.modules[__name__].__class__ = _CallableModule
