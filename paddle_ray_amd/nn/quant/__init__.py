"""paddle.nn.quant (parity: python/paddle/nn/quant/): fake-quant layers, quantized layer
wrappers, QAT layers, stubs and the ONNX-style quantize/dequantize format layers."""
from .functional_layers import (FloatFunctionalLayer, add, subtract, multiply, divide,  # noqa
                                reshape, transpose, concat, flatten, matmul)
from .quant_layers import (FakeQuantAbsMax, FakeQuantMovingAverageAbsMax,  # noqa: F401
                           FakeQuantChannelWiseAbsMax, MovingAverageAbsMaxScale, QuantizedConv2D,
                           QuantizedConv2DTranspose, QuantizedLinear, QuantizedMatmul,
                           QuantizedColumnParallelLinear, QuantizedRowParallelLinear,
                           MAOutputScaleLayer, FakeQuantMAOutputScaleLayer, QuantStub)
from .format import (LinearQuanter, LinearDequanter, LinearQuanterDequanter,  # noqa: F401
                     ConvertibleQuantedLayer)
from .stub import Stub, QuanterStub  # noqa: F401
from .lsq import FakeQuantActLSQPlus, FakeQuantWeightLSQPlus  # noqa: F401
from . import qat  # noqa: F401

__all__ = ['Stub']
