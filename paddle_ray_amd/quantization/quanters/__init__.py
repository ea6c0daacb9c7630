"""Built-in quanters (parity: python/paddle/quantization/quanters/abs_max.py)."""
import torch

from ...framework.core import Tensor, _u
from ...ops import quant as Q
from ..base import BaseQuanter, QuanterFactory


class FakeQuanterWithAbsMaxObserver(QuanterFactory):
    """Moving-average abs-max fake quanter factory:
    state = rate*state + 1; accum = rate*accum + max|x|; scale = accum / state.
    ``fp8=True`` simulates OCP float8 e4m3 instead of ``bit_length``-bit integers."""

    def __init__(self, moving_rate=0.9, bit_length=8, dtype='float32', name=None, fp8=False):
        super().__init__(name=name, moving_rate=moving_rate, bit_length=bit_length, dtype=dtype,
                         fp8=fp8)

    def _get_class(self):
        return FakeQuanterWithAbsMaxObserverLayer


class FakeQuanterWithAbsMaxObserverLayer(BaseQuanter):
    def __init__(self, layer, name=None, moving_rate=0.9, bit_length=8, dtype='float32',
                 fp8=False):
        super().__init__()
        from ...nn.quant.quant_layers import _param
        self._moving_rate, self._bit_length, self._fp8 = moving_rate, bit_length, fp8
        self._scale = _param(self, [1], 0.001, dtype)
        self._state = _param(self, [1], 1.0, dtype)
        self._accum = _param(self, [1], 1.0, dtype)

    def forward(self, input):
        x = _u(input)
        if self.training:
            s = Q.moving_average_update(_u(self._state), _u(self._accum), Q.absmax(x),
                                        self._moving_rate)
            with torch.no_grad():
                _u(self._scale).copy_(s)
        return Tensor(Q.fake_quant_dequant(x, _u(self._scale)[0], self._bit_length,
                                           fp8=self._fp8))

    def bit_length(self):
        return self._bit_length

    def quant_axis(self):
        return None

    def scales(self):
        return self._scale

    def zero_points(self):
        return None


__all__ = ['FakeQuanterWithAbsMaxObserver']
