"""PHI-equivalent kernel registry (parity: paddle/phi/core/kernel_registry.h, kernel_factory.cc).

Kernels are keyed by ``(op_name, backend)`` with backend in {'hip', 'ref'}.
``hip`` kernels are the hand-written gfx950 kernels in ``ops/csrc`` (loaded from
the in-tree ``_pra_hip`` extension); ``ref`` kernels are PyTorch compositions
used on CPU and as numerics references in tests. On a GPU tensor the registry
picks ``hip``; if the native library is missing on a machine that HAS a GPU it
raises instead of silently falling back (set ``PRA_ALLOW_REF=1`` to opt out,
e.g. for A/B ablations).
"""
import collections
import os

import torch

from ..framework import nan_inf as _nan_inf

_KERNELS = {}
_STATS = collections.Counter()
_FORCE_REF = os.environ.get('PRA_FORCE_REF', '0') == '1'
_ALLOW_REF = os.environ.get('PRA_ALLOW_REF', '0') == '1'


def register_kernel(op, backend):
    def deco(fn):
        _KERNELS[(op, backend)] = fn
        return fn
    return deco


def has_kernel(op, backend):
    return (op, backend) in _KERNELS


def get_kernel(op, backend):
    return _KERNELS[(op, backend)]


def list_kernels():
    return sorted(_KERNELS)


def select_backend(t: torch.Tensor, op=None):
    """'hip' for device tensors (native lib required), 'ref' for host tensors."""
    if t.is_cuda and not _FORCE_REF:
        from . import _native
        if _native.available():
            if op is None or (op, 'hip') in _KERNELS:
                _STATS[(op, 'hip')] += 1
                return 'hip'
        elif not _ALLOW_REF:
            _native.require()  # raises with the load error
    _STATS[(op, 'ref')] += 1
    return 'ref'


def dispatch(op, t, *args, **kwargs):
    out = _KERNELS[(op, select_backend(t, op))](*args, **kwargs)
    if _nan_inf._state['mode'] is not None:
        _nan_inf.check_outputs(op, out)
    return out


def stats():
    return dict(_STATS)


def reset_stats():
    _STATS.clear()
