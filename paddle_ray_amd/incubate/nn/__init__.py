"""paddle.incubate.nn fused layers (parity: python/paddle/incubate/nn/layer/fused_transformer.py)."""
from . import functional  # noqa
from .layer import (FusedMultiHeadAttention, FusedFeedForward, FusedTransformerEncoderLayer,  # noqa
                    FusedMultiTransformer, FusedLinear, FusedBiasDropoutResidualLayerNorm,
                    FusedEcMoe, FusedDropoutAdd)
