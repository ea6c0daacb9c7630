"""Mixture-of-Experts with expert parallelism (parity:
python/paddle/incubate/distributed/models/moe/)."""
from .gate import BaseGate, NaiveGate, GShardGate, SwitchGate  # noqa: F401
from .moe_layer import MoELayer  # noqa: F401
from .grad_clip import ClipGradForMOEByGlobalNorm  # noqa: F401
