"""paddle.incubate.tensor import path (reference python/paddle/incubate/tensor/math.py): the
segment reductions of paddle.geometric."""
from ...geometric import segment_sum, segment_mean, segment_max, segment_min  # noqa: F401

__all__ = []
