"""Static-graph placeholder API surface; the full Program/Executor lives in static/graph.py."""
from . import _STATIC


def enable_static():
    _STATIC[0] = True


def disable_static(place=None):
    _STATIC[0] = False


def _static_minimize(opt, loss, parameters=None):
    raise NotImplementedError("static minimize")
