"""fleet.layers.mpu (parity: python/paddle/distributed/fleet/layers/mpu/__init__.py)."""
from .....parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear,  # noqa
                                          VocabParallelEmbedding, ParallelCrossEntropy,
                                          get_rng_state_tracker, model_parallel_random_seed,
                                          _c_identity, _mp_allreduce, _c_split, _c_concat, split)
from .....parallel.tensor_parallel import RNGStatesTracker  # noqa
mp_ops = None
