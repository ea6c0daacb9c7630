"""paddle.distributed.fleet.dataset import path (reference python/paddle/distributed/fleet/
dataset/__init__.py): the file datasets of distributed/dataset.py."""
from ...dataset import InMemoryDataset, QueueDataset  # noqa: F401
from ...dataset import _FileDataset as DatasetBase  # noqa: F401

__all__ = []
