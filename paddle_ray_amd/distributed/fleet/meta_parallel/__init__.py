"""fleet.meta_parallel (parity: python/paddle/distributed/fleet/meta_parallel/__init__.py)."""
from ....parallel.pipeline import (LayerDesc, SharedLayerDesc, PipelineLayer,  # noqa
                                   PipelineParallel, SegmentLayers)
from ....parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear,  # noqa
                                          VocabParallelEmbedding, ParallelCrossEntropy,
                                          get_rng_state_tracker, model_parallel_random_seed,
                                          RNGStatesTracker)
from .. import TensorParallel  # noqa
from ....parallel.sharding import ShardedModel as GroupShardedStage3  # noqa
from ....parallel.sharding import ShardedModel as GroupShardedStage2  # noqa
from ....parallel.sharding import ShardedOptimizer as GroupShardedOptimizerStage2  # noqa
