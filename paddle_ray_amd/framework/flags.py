"""Global FLAGS registry (parity: paddle.set_flags/get_flags, paddle/phi/core/flags.cc).

Flags are seeded from ``FLAGS_*`` environment variables at import.
Recognised: FLAGS_check_nan_inf (NaN/Inf checker on layer outputs and grads),
FLAGS_cudnn_deterministic, FLAGS_eager_delete_tensor_gb, FLAGS_allocator_strategy,
FLAGS_fraction_of_gpu_memory_to_use, FLAGS_call_stack_level, FLAGS_use_hip_kernels,
FLAGS_cudnn_exhaustive_search (MIOpen find-mode conv algorithm search, cached per shape).
"""
import os

_FLAGS = {
    'FLAGS_check_nan_inf': False,
    'FLAGS_check_nan_inf_level': 0,
    'FLAGS_cudnn_deterministic': False,
    'FLAGS_eager_delete_tensor_gb': 0.0,
    'FLAGS_allocator_strategy': 'auto_growth',
    'FLAGS_fraction_of_gpu_memory_to_use': 0.92,
    'FLAGS_call_stack_level': 1,
    'FLAGS_use_hip_kernels': True,
    'FLAGS_embedding_deterministic': 0,
    'FLAGS_benchmark': False,
    'FLAGS_cudnn_exhaustive_search': False,
}


def _parse(v, like):
    if isinstance(like, bool):
        return str(v).lower() in ('1', 'true', 'yes', 'on')
    if isinstance(like, int):
        return int(v)
    if isinstance(like, float):
        return float(v)
    return v


for _k in list(_FLAGS):
    if _k in os.environ:
        _FLAGS[_k] = _parse(os.environ[_k], _FLAGS[_k])


def set_flags(flags):
    for k, v in flags.items():
        if not k.startswith('FLAGS_'):
            k = 'FLAGS_' + k
        _FLAGS[k] = v
        if k == 'FLAGS_cudnn_deterministic':
            import torch
            torch.backends.cudnn.deterministic = bool(v)
        if k == 'FLAGS_cudnn_exhaustive_search':
            import torch
            torch.backends.cudnn.benchmark = bool(v)
        if k in ('FLAGS_check_nan_inf', 'FLAGS_check_nan_inf_level'):
            _apply_nan_inf()


def _apply_nan_inf():
    from . import nan_inf
    if _FLAGS['FLAGS_check_nan_inf']:
        nan_inf.enable(_FLAGS['FLAGS_check_nan_inf_level'])
    else:
        nan_inf.disable()


def get_flags(flags):
    if isinstance(flags, str):
        flags = [flags]
    out = {}
    for k in flags:
        kk = k if k.startswith('FLAGS_') else 'FLAGS_' + k
        if kk not in _FLAGS:
            raise ValueError(f"unknown flag {k}")
        out[k] = _FLAGS[kk]
    return out


def flag(name):
    return _FLAGS.get(name)


if _FLAGS['FLAGS_check_nan_inf']:
    _apply_nan_inf()
