"""paddle.cost_model (parity: python/paddle/cost_model/__init__.py)."""
from .cost_model import CostModel  # noqa: F401

__all__ = []
