"""PHI-equivalent kernel registry (parity: paddle/phi/core/kernel_registry.h, kernel_factory.cc).

Kernels are keyed by ``(op_name, backend, dtype)`` with backend in {'hip', 'ref'} and dtype
a torch dtype or ``None`` (any dtype) — the analogue of PHI's KernelKey (backend, layout,
dtype); layouts here are always dense row-major. Dispatch picks the exact dtype of the
selector tensor first, then the any-dtype kernel; a HIP kernel registered only for some dtypes
is never handed another one (the op runs its ``ref`` kernel instead, visible in ``stats()``).
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


def register_kernel(op, backend, dtypes=None):
    """Register ``fn`` for ``(op, backend)`` and each of ``dtypes`` (None = any dtype)."""
    def deco(fn):
        tab = _KERNELS.setdefault((op, backend), {})
        for d in (tuple(dtypes) if dtypes else (None,)):
            tab[d] = fn
        return fn
    return deco


def _lookup(op, backend, dtype):
    tab = _KERNELS.get((op, backend))
    if not tab:
        return None
    fn = tab.get(dtype)
    return fn if fn is not None else tab.get(None)


def has_kernel(op, backend, dtype=None):
    tab = _KERNELS.get((op, backend), {})
    return (dtype in tab or None in tab) if dtype is not None else bool(tab)


def get_kernel(op, backend, dtype=None):
    fn = _lookup(op, backend, dtype)
    if fn is None:
        tab = _KERNELS.get((op, backend), {})
        if dtype is None and tab:
            return next(iter(tab.values()))
        raise KeyError(f"no {backend} kernel for op {op!r} dtype {dtype}")
    return fn


def list_kernels():
    return sorted(_KERNELS)


def kernel_table():
    """{(op, backend): [dtype names]} — the registered kernel keys."""
    return {k: sorted('any' if d is None else str(d).replace('torch.', '') for d in v)
            for k, v in sorted(_KERNELS.items())}


def select_backend(t: torch.Tensor, op=None):
    """'hip' for device tensors whose dtype has a HIP kernel (native lib required), else
    'ref'."""
    if t.is_cuda and not _FORCE_REF:
        from . import _native
        if _native.available():
            if op is None or _lookup(op, 'hip', t.dtype) is not None:
                _STATS[(op, 'hip')] += 1
                return 'hip'
        elif not _ALLOW_REF:
            _native.require()  # raises with the load error
    if op is not None and (op, 'ref') not in _KERNELS and (op, 'hip') in _KERNELS:
        _STATS[(op, 'hip')] += 1  # device-only op (e.g. multi-tensor optimizer tables)
        return 'hip'
    _STATS[(op, 'ref')] += 1
    return 'ref'


def dispatch(op, t, *args, **kwargs):
    backend = select_backend(t, op)
    out = get_kernel(op, backend, t.dtype)(*args, **kwargs)
    if _nan_inf._state['mode'] is not None:
        _nan_inf.check_outputs(op, out)
    return out


def stats():
    return dict(_STATS)


def reset_stats():
    _STATS.clear()
