import collections
import contextlib

_counters = collections.defaultdict(int)


def generate(key):
    n = _counters[key]
    _counters[key] += 1
    return f'{key}_{n}'


@contextlib.contextmanager
def guard(new_generator=None):
    global _counters
    old = _counters
    _counters = collections.defaultdict(int)
    try:
        yield
    finally:
        _counters = old
