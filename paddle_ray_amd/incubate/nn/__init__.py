"""paddle.incubate.nn fused layers (parity: python/paddle/incubate/nn/layer/fused_transformer.py)."""
from . import functional  # noqa
from .layer import (FusedMultiHeadAttention, FusedFeedForward, FusedTransformerEncoderLayer,  # noqa
                    FusedMultiTransformer, FusedMultiTransformerDecoder, FusedLinear, FusedBiasDropoutResidualLayerNorm,
                    FusedEcMoe, FusedDropoutAdd)
from . import attn_bias  # noqa: E402,F401
from .memory_efficient_attention import memory_efficient_attention  # noqa: E402,F401
from .loss import identity_loss  # noqa: E402,F401
