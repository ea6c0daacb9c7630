"""fleet.utils (parity: python/paddle/distributed/fleet/utils/__init__.py)."""
from ....parallel.recompute import recompute  # noqa
from . import hybrid_parallel_util  # noqa
from .fs import LocalFS, HDFSClient  # noqa
from .ps_util import DistributedInfer  # noqa
