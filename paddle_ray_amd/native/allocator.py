"""Native auto-growth best-fit device allocator (native/alloc/auto_growth_allocator.cpp).

Parity: the reference's FLAGS_allocator_strategy='auto_growth' allocator
(paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc) with stream-safe reuse
(stream_safe_cuda_allocator.cc). It is the default on a GPU host (installed when
paddle_ray_amd is imported, before the first device allocation; ``PRA_ALLOCATOR=caching``
opts out), or ``enable()`` before any GPU tensor exists; it then backs every PyTorch-ROCm tensor through
``torch.cuda.memory.CUDAPluggableAllocator``. ``PRA_ALLOC_CHUNK_MB`` sets the growth chunk
(default 64 MB). HIP-graph capture: the allocator is installed through the C++ hooks
(alloc/torch_hooks.cpp, ``_pra_alloc_torch``), which route every allocation made on a capturing
stream into a private arena per graph pool (released with the graph), so captured graphs never
share memory with eager code. Without that module (ctypes-only pluggable allocator) enabling
refuses, since captures would be unsafe. ``Tensor.record_stream`` is honoured: a block freed
while other streams recorded on it is held back until events recorded on those streams at free
time complete (as PyTorch's caching allocator does; RCCL's stream use depends on it).
Measured against PyTorch's caching allocator (profiles/r3h/ab_results.txt, profiles/r3j/):
GPT-1.3B 124.2K vs 124.4K tokens/s, ResNet-50 8431 vs 8423 img/s, BERT-base (HIP-graph static
executor) 1698.6 vs 1697.4 seq/s (an earlier 1473 vs 1592 gap is gone since the Executor hands
captured gradients to the optimizer in place).
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
    if not host:
        lib.pra_alloc_pool.restype = ctypes.c_void_p
        lib.pra_alloc_pool.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_uint64]
        lib.pra_pool_release.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
    lib.pra_pool_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
    lib.pra_record_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return lib


def hooks():
    """The C++ PyTorch integration (graph-capture pools), or None when it is not built."""
    try:
        from . import _pra_alloc_torch
        return _pra_alloc_torch
    except ImportError:
        return None


def enable():
    """Route every device allocation of this process through the native allocator (graph
    captures into per-pool arenas). Must run before the first device allocation."""
    if _state['enabled']:
        return True
    h = hooks()
    if h is None:
        raise RuntimeError('native allocator: _pra_alloc_torch (graph-pool hooks) is not built; '
                           'run python -m paddle_ray_amd.native.build')
    lib = load()
    addr = [ctypes.cast(getattr(lib, n), ctypes.c_void_p).value
            for n in ('pra_alloc', 'pra_free', 'pra_alloc_pool', 'pra_pool_release', 'pra_record_stream')]
    if not h.install(*addr):
        raise RuntimeError('native allocator: torch rejected the pluggable allocator')
    _state['lib'] = lib
    _state['enabled'] = True
    return True


def enabled():
    return _state['enabled']


def stats(device=0, lib=None):
    lib = lib or _state['lib']
    buf = (ctypes.c_int64 * 9)()
    lib.pra_alloc_stats(int(device), buf)
    d = dict(zip(_STAT_NAMES, list(buf)))
    pb = (ctypes.c_int64 * 3)()
    lib.pra_pool_stats(int(device), pb)
    d['pool_allocated'], d['pool_reserved'], d['num_pools'] = list(pb)
    return d


def empty_cache(device=0, lib=None):
    return int((lib or _state['lib']).pra_alloc_empty_cache(int(device)))


def reset_peak(device=0, lib=None):
    (lib or _state['lib']).pra_alloc_reset_peak(int(device))


def maybe_enable_from_env():
    """The native allocator is the DEFAULT on a GPU host (reference default
    FLAGS_allocator_strategy=auto_growth, paddle/phi/core/flags.cc:489). Opt out with
    ``PRA_ALLOCATOR=caching`` (or ``FLAGS_allocator_strategy=naive_best_fit``): PyTorch's caching
    allocator. No GPU, or the graph-pool hooks not built: the caching allocator, with a warning
    in the latter case. Runs at import, before any device allocation (device_count() does not
    initialise the GPU)."""
    choice = os.environ.get('PRA_ALLOCATOR', '').strip().lower()
    strat = os.environ.get('FLAGS_allocator_strategy', '').strip().lower()
    if choice in ('caching', 'torch', 'off', '0') or (not choice and strat == 'naive_best_fit'):
        return False
    if os.environ.get('PRA_FORCE_CPU') == '1':
        return False
    try:
        import torch
        if torch.cuda.device_count() == 0:
            return False
    except Exception:
        return False
    if choice in ('auto_growth', 'native'):
        return enable()   # explicitly requested: fail loudly
    if hooks() is None or not os.path.exists(library_path()):
        import warnings
        warnings.warn('native allocator not built (python -m paddle_ray_amd.native.build): '
                      'using the PyTorch caching allocator')
        return False
    return enable()
