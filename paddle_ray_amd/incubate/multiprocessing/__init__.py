"""paddle.incubate.multiprocessing (parity: python/paddle/incubate/multiprocessing/).

``multiprocessing`` with reductions registered so framework Tensors (CPU: shared memory;
device: HIP IPC through torch's dmabuf-based CUDA-IPC reductions) can be passed through
queues / pipes between processes without copying."""
import multiprocessing
from multiprocessing import *  # noqa: F401,F403

from .reductions import init_reductions

__all__ = []

init_reductions()
