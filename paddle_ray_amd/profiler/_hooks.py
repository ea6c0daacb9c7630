"""Cheap profiler switches read on hot paths (Layer.__call__, Tensor.backward, optimizers,
collectives, DataLoader): ``ACTIVE`` is non-empty only while some Profiler records."""
import threading

ACTIVE = []            # recording Profiler objects
_tls = threading.local()


def layer_depth():
    return getattr(_tls, 'depth', 0)


def enter_layer():
    _tls.depth = getattr(_tls, 'depth', 0) + 1


def exit_layer():
    _tls.depth = getattr(_tls, 'depth', 1) - 1
