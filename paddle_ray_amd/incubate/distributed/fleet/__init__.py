"""paddle.incubate.distributed.fleet (parity: python/paddle/incubate/distributed/fleet/
__init__.py): the recompute helpers for Sequential models and hybrid-parallel layers."""
from ....parallel.recompute import recompute_sequential, recompute_hybrid  # noqa: F401

__all__ = ['recompute_sequential', 'recompute_hybrid']
