"""paddle.reader (parity: python/paddle/reader/__init__.py)."""
from .decorator import (map_readers, shuffle, xmap_readers, firstn, buffered,  # noqa: F401
                        compose, cache, ComposeNotAligned, chain, multiprocess_reader)

__all__ = []
