"""auto_parallel.Strategy (parity: reference python/paddle/distributed/auto_parallel/strategy.py
and constants.py: sections with an `enable` switch and their fields; dict or attribute access)."""
import copy

_DEFAULTS = {
    'auto_mode': 'semi',
    'gradient_scale': True,
    'use_cache': True,
    'return_numpy': True,
    'all_ranks': False,
    'split_data': True,
    'seed': None,
    'recompute': {'enable': False, 'checkpoints': [], 'no_recompute_segments': []},
    'amp': {'enable': False, 'dtype': 'bfloat16', 'level': 'o1', 'init_loss_scaling': 32768.0,
            'incr_every_n_steps': 1000, 'decr_every_n_nan_or_inf': 2, 'incr_ratio': 2.0,
            'decr_ratio': 0.8, 'use_dynamic_loss_scaling': True, 'custom_white_list': [],
            'custom_black_list': [], 'use_master_grad': False},
    'sharding': {'enable': False, 'stage': 1, 'degree': 8, 'enable_overlap': False},
    'gradient_merge': {'enable': False, 'k_steps': 1, 'avg': True},
    'pipeline': {'enable': False, 'schedule_mode': '1F1B', 'micro_batch_size': 1,
                 'accumulate_steps': 1},
    'qat': {'enable': False},
    'tuning': {'enable': False},
    'dataset': {'enable': False, 'num_shards': 1},
    'fused_passes': {'enable': False, 'fused_passes_list': []},
}


class _Section:
    def __init__(self, name, values):
        self.__dict__['_name'] = name
        self.__dict__['_values'] = dict(values)

    def __getattr__(self, k):
        try:
            return self.__dict__['_values'][k]
        except KeyError:
            raise AttributeError(f"{self._name} has no field {k!r}") from None

    def __setattr__(self, k, v):
        if k not in self._values:
            raise AttributeError(f"{self._name} has no field {k!r}")
        self._values[k] = v

    def to_dict(self):
        return dict(self._values)

    def __repr__(self):
        return f"{self._name}: {self._values}"


class Strategy:
    def __init__(self, config=None):
        config = dict(config or {})
        for k, v in _DEFAULTS.items():
            if isinstance(v, dict):
                vals = copy.deepcopy(v)
                vals.update(config.pop(k, {}) or {})
                object.__setattr__(self, k, _Section(k, vals))
            else:
                object.__setattr__(self, k, config.pop(k, v))
        if config:
            raise ValueError(f"unknown Strategy fields: {sorted(config)}")

    def __setattr__(self, k, v):
        if k not in _DEFAULTS:
            raise AttributeError(f"Strategy has no field {k!r}")
        if isinstance(_DEFAULTS[k], dict):
            raise AttributeError(f"set fields of strategy.{k} instead")
        object.__setattr__(self, k, v)

    def to_dict(self):
        return {k: (getattr(self, k).to_dict() if isinstance(v, dict) else getattr(self, k))
                for k, v in _DEFAULTS.items()}

    def __deepcopy__(self, memo):
        return Strategy(self.to_dict())

    def __repr__(self):
        return f"Strategy({self.to_dict()})"
