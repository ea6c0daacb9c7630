"""paddle.distributed.parallel (parity: python/paddle/distributed/parallel.py)."""
from ..parallel.data_parallel import DataParallel  # noqa
from .collective import init_parallel_env, ParallelEnv, get_rank, get_world_size  # noqa
