"""paddle.geometric.sampling import path (reference python/paddle/geometric/sampling/
neighbors.py)."""
from .. import sample_neighbors, weighted_sample_neighbors  # noqa: F401

__all__ = []
