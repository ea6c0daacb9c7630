"""paddle.nn (parity: python/paddle/nn/__init__.py)."""
from . import functional, initializer  # noqa
from .layer.layers import Layer, ParamAttr, WeightNormParamAttr  # noqa
from .layer.common import (Identity, Linear, Bilinear, Embedding, Dropout, Dropout2D, Dropout3D,  # noqa
                           AlphaDropout, Flatten, Unflatten, Upsample, UpsamplingNearest2D,
                           UpsamplingBilinear2D, Pad1D, Pad2D, Pad3D, ZeroPad2D, CosineSimilarity,
                           PairwiseDistance, Unfold, Fold, PixelShuffle, PixelUnshuffle,
                           ChannelShuffle, ReLU, ReLU6, LeakyReLU, ELU, CELU, SELU, GELU, Silu, Swish,
                           Mish, Sigmoid, Tanh, Hardtanh, Hardsigmoid, Hardswish, Hardshrink,
                           Softshrink, Softsign, Softplus, Tanhshrink, ThresholdedReLU, LogSigmoid,
                           Softmax, LogSoftmax, Maxout, GLU, RReLU, Softmax2D, PReLU, Sequential,
                           LayerList, LayerDict, ParameterList)
from .layer.norm import (LayerNorm, RMSNorm, BatchNorm, BatchNorm1D, BatchNorm2D, BatchNorm3D,  # noqa
                         SyncBatchNorm, InstanceNorm1D, InstanceNorm2D, InstanceNorm3D, GroupNorm,
                         LocalResponseNorm, SpectralNorm)
from .layer.conv import (Conv1D, Conv2D, Conv3D, Conv1DTranspose, Conv2DTranspose,  # noqa
                         Conv3DTranspose, MaxPool1D, MaxPool2D, MaxPool3D, AvgPool1D, AvgPool2D,
                         AvgPool3D, AdaptiveAvgPool1D, AdaptiveAvgPool2D, AdaptiveAvgPool3D,
                         AdaptiveMaxPool1D, AdaptiveMaxPool2D, AdaptiveMaxPool3D, MaxUnPool1D,
                         MaxUnPool2D, MaxUnPool3D)
from .layer.loss import *  # noqa
from .layer.transformer import (MultiHeadAttention, TransformerEncoderLayer, TransformerEncoder,  # noqa
                                TransformerDecoderLayer, TransformerDecoder, Transformer)
from .layer.rnn import (RNNCellBase, SimpleRNNCell, LSTMCell, GRUCell, RNN, BiRNN, SimpleRNN,  # noqa
                        LSTM, GRU)
from .clip import ClipGradByValue, ClipGradByNorm, ClipGradByGlobalNorm  # noqa
from . import utils  # noqa
from .decode import BeamSearchDecoder, dynamic_decode, Decoder  # noqa: E402
from . import quant  # noqa: E402
