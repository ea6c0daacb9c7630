"""paddle.distributed (parity: python/paddle/distributed/__init__.py)."""
from .collective import (ReduceOp, Group, ParallelEnv, init_parallel_env, is_initialized,  # noqa
                         is_available, new_group, get_group, destroy_process_group, get_rank,
                         get_world_size, get_backend, all_reduce, broadcast, reduce, all_gather,
                         all_gather_into_tensor, all_gather_object, broadcast_object_list,
                         scatter_object_list, reduce_scatter, scatter, alltoall, alltoall_single,
                         send, recv, isend, irecv, P2POp, batch_isend_irecv, barrier, wait, split,
                         gloo_init_parallel_env, gloo_barrier, gloo_release)
from .parallel import DataParallel  # noqa
from . import sharding  # noqa
from . import fleet  # noqa
from .spawn import spawn  # noqa
from . import launch  # noqa
from .dataset import InMemoryDataset, QueueDataset  # noqa
from .entry_attr import ProbabilityEntry, CountFilterEntry, ShowClickEntry  # noqa


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3


from . import io  # noqa
from . import watchdog  # noqa: E402
from . import models  # noqa: E402
from . import utils  # noqa: E402
from . import rpc  # noqa: E402
from . import communication  # noqa: E402
from . import auto_parallel  # noqa: E402
from . import passes  # noqa: E402
from .auto_parallel import ProcessMesh, shard_tensor, shard_op, reshard, Strategy, Engine  # noqa: E402
