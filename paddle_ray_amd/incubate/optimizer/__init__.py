"""paddle.incubate.optimizer (parity: python/paddle/incubate/optimizer/{lookahead,
modelaverage,distributed_fused_lamb,lbfgs}.py and functional/{bfgs,lbfgs}.py)."""
from .lookahead import LookAhead  # noqa: F401
from .modelaverage import ModelAverage  # noqa: F401
from .distributed_fused_lamb import DistributedFusedLamb  # noqa: F401
from .lbfgs import LBFGS  # noqa: F401
from . import functional  # noqa: F401
