"""Native auto-growth best-fit device allocator (native/alloc/auto_growth_allocator.cpp).

Parity: the reference's FLAGS_allocator_strategy='auto_growth' allocator
(paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc) with stream-safe reuse
(stream_safe_cuda_allocator.cc). Enable it for a process with ``PRA_ALLOCATOR=auto_growth``
(read when paddle_ray_amd is imported, before the first device allocation) or by calling
``enable()`` before any GPU tensor exists; it then backs every PyTorch-ROCm tensor through
``torch.cuda.memory.CUDAPluggableAllocator``. ``PRA_ALLOC_CHUNK_MB`` sets the growth chunk
(default 64 MB). Limitation: PyTorch's pluggable-allocator hook has no ``record_stream``, so
a tensor freed while a SIDE stream still uses it must be synchronised by its owner (the
framework's own collectives wait on their works before buffers are released).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_state = {'enabled': False, 'lib': None}
_STAT_NAMES = ('allocated', 'reserved', 'peak_allocated', 'peak_reserved', 'num_allocs',
               'num_frees', 'num_chunks', 'num_backend_allocs', 'num_backend_frees')


def library_path(host=False):
    return os.path.join(_HERE, '_pra_alloc_host.so' if host else '_pra_alloc_hip.so')


def load(host=False):
    lib = ctypes.CDLL(library_path(host))
    lib.pra_alloc.restype = ctypes.c_void_p
    lib.pra_alloc.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    lib.pra_free.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    lib.pra_alloc_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
    lib.pra_alloc_empty_cache.restype = ctypes.c_int64
    lib.pra_alloc_empty_cache.argtypes = [ctypes.c_int]
    lib.pra_alloc_reset_peak.argtypes = [ctypes.c_int]
    lib.pra_alloc_set_growth.argtypes = [ctypes.c_int, ctypes.c_int64]
    lib.pra_alloc_check.argtypes = [ctypes.c_int]
    return lib


def enable():
    """Route every device allocation of this process through the native allocator."""
    if _state['enabled']:
        return True
    import torch
    alloc = torch.cuda.memory.CUDAPluggableAllocator(library_path(), 'pra_alloc', 'pra_free')
    torch.cuda.memory.change_current_allocator(alloc)
    _state['lib'] = load()
    _state['enabled'] = True
    return True


def enabled():
    return _state['enabled']


def stats(device=0, lib=None):
    lib = lib or _state['lib']
    buf = (ctypes.c_int64 * 9)()
    lib.pra_alloc_stats(int(device), buf)
    return dict(zip(_STAT_NAMES, list(buf)))


def empty_cache(device=0, lib=None):
    return int((lib or _state['lib']).pra_alloc_empty_cache(int(device)))


def reset_peak(device=0, lib=None):
    (lib or _state['lib']).pra_alloc_reset_peak(int(device))


def maybe_enable_from_env():
    if os.environ.get('PRA_ALLOCATOR', '') in ('auto_growth', 'native'):
        enable()
