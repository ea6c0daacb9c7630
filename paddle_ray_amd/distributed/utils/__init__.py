"""paddle.distributed.utils (parity: python/paddle/distributed/utils/)."""
from . import moe_utils  # noqa: F401
from .moe_utils import global_scatter, global_gather  # noqa: F401
