"""MI355X parallel runtime: flat buffers, DP, ZeRO sharding, TP, PP, recompute, hybrid topology."""
from .flat import FlatGroup, group_params_into_buckets  # noqa
from .data_parallel import DataParallel, GradBucketReducer  # noqa
from .sharding import (group_sharded_parallel, save_group_sharded_model, ShardedModel,  # noqa
                       ShardedOptimizer, ShardedState)
