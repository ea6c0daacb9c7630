"""paddle.distributed.models (parity: python/paddle/distributed/models/)."""
from . import moe  # noqa: F401
