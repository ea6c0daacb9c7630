"""paddle.device.cuda — HIP streams/events/memory stats on MI355X (parity: python/paddle/device/cuda/__init__.py).

Memory stats come from the PyTorch-ROCm caching allocator (HBM3E, 288 GB per GPU).
"""
import contextlib

import torch


def _dev(device):
    if device is None:
        return torch.cuda.current_device()
    if isinstance(device, int):
        return device
    s = str(device)
    return int(s.split(':')[1]) if ':' in s else 0


def device_count():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def synchronize(device=None):
    torch.cuda.synchronize(_dev(device))


def _native():
    from ...native import allocator
    return allocator if allocator.enabled() else None


def _idx(device):
    d = _dev(device)
    return d.index if isinstance(d, torch.device) and d.index is not None else \
        (d if isinstance(d, int) else torch.cuda.current_device())


def _nstat(device, key):
    return _native().stats(_idx(device))[key]


def empty_cache():
    if _native():
        _native().empty_cache(torch.cuda.current_device())
        return
    torch.cuda.empty_cache()


def max_memory_allocated(device=None):
    if _native():
        return _nstat(device, 'peak_allocated')
    return torch.cuda.max_memory_allocated(_dev(device))


def max_memory_reserved(device=None):
    if _native():
        return _nstat(device, 'peak_reserved')
    return torch.cuda.max_memory_reserved(_dev(device))


def memory_allocated(device=None):
    if _native():
        return _nstat(device, 'allocated')
    return torch.cuda.memory_allocated(_dev(device))


def memory_reserved(device=None):
    if _native():
        return _nstat(device, 'reserved')
    return torch.cuda.memory_reserved(_dev(device))


def reset_max_memory_allocated(device=None):
    if _native():
        _native().reset_peak(_idx(device))
        return
    torch.cuda.reset_peak_memory_stats(_dev(device))


def get_device_properties(device=None):
    return torch.cuda.get_device_properties(_dev(device))


def get_device_name(device=None):
    return torch.cuda.get_device_name(_dev(device))


def get_device_capability(device=None):
    return torch.cuda.get_device_capability(_dev(device))


class Stream:
    def __init__(self, device=None, priority=2):
        self._s = torch.cuda.Stream(device=_dev(device) if device is not None else None,
                                    priority=-1 if priority == 1 else 0)

    def wait_event(self, event):
        self._s.wait_event(event._e)

    def wait_stream(self, stream):
        self._s.wait_stream(stream._s if isinstance(stream, Stream) else stream)

    def record_event(self, event=None):
        event = event or Event()
        event._e.record(self._s)
        return event

    def query(self):
        return self._s.query()

    def synchronize(self):
        self._s.synchronize()

    @property
    def cuda_stream(self):
        return self._s.cuda_stream


class Event:
    def __init__(self, enable_timing=False, blocking=False, interprocess=False):
        self._e = torch.cuda.Event(enable_timing=enable_timing, blocking=blocking,
                                   interprocess=interprocess)

    def record(self, stream=None):
        self._e.record(None if stream is None else (stream._s if isinstance(stream, Stream)
                                                   else stream))

    def query(self):
        return self._e.query()

    def synchronize(self):
        self._e.synchronize()

    def elapsed_time(self, end_event):
        return self._e.elapsed_time(end_event._e)


def current_stream(device=None):
    s = Stream.__new__(Stream)
    s._s = torch.cuda.current_stream(_dev(device) if device is not None else None)
    return s


def set_stream(stream):
    """Make ``stream`` the current stream of its device; returns the previous current stream
    (parity: python/paddle/device/__init__.py:900 set_stream)."""
    ts = stream._s if isinstance(stream, Stream) else stream
    prev = current_stream(ts.device)
    torch.cuda.set_stream(ts)
    return prev


@contextlib.contextmanager
def stream_guard(stream):
    with torch.cuda.stream(stream._s if isinstance(stream, Stream) else stream):
        yield
