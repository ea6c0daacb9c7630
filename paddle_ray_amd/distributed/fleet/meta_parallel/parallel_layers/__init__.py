"""paddle.distributed.fleet.meta_parallel.parallel_layers import path (reference
meta_parallel/parallel_layers/{mp_layers,pp_layers,random}.py): the tensor-parallel layers,
pipeline layer descriptions and the model-parallel RNG tracker of parallel/."""
from .. import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,  # noqa: F401
                ParallelCrossEntropy, LayerDesc, SharedLayerDesc, PipelineLayer,
                get_rng_state_tracker, model_parallel_random_seed, RNGStatesTracker)

__all__ = []
