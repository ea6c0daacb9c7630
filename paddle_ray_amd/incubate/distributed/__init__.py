"""paddle.incubate.distributed (parity: python/paddle/incubate/distributed/)."""
from . import models  # noqa: F401
from . import fleet  # noqa: F401
