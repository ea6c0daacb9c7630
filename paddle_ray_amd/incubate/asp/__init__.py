"""paddle.incubate.asp (parity: python/paddle/incubate/asp/__init__.py)."""
from .utils import (calculate_density, check_mask_1d, get_mask_1d, check_mask_2d,  # noqa
                    get_mask_2d_greedy, get_mask_2d_best, create_mask, check_sparsity,
                    MaskAlgo, CheckMethod)
from .asp import (decorate, prune_model, set_excluded_layers, reset_excluded_layers,  # noqa
                  add_supported_layer)

__all__ = ['calculate_density', 'decorate', 'prune_model', 'set_excluded_layers',
           'reset_excluded_layers', 'add_supported_layer']
