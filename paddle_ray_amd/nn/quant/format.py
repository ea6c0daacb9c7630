"""ONNX-style quantize / dequantize layers and the convertible-quanted-layer protocol
(parity: python/paddle/nn/quant/format.py)."""
import abc

import torch

from ...framework.core import Tensor, _u
from ...ops import quant as Q
from ..layer.layers import Layer


def _as_t(v):
    if v is None:
        return None
    if isinstance(v, Tensor):
        return _u(v).detach().float()
    return torch.as_tensor(v, dtype=torch.float32)


class LinearQuanter(Layer):
    """x -> clip(round(x / scale * range), -range-1, range) (float-held integers)."""

    def __init__(self, scales, zero_point=None, quant_axis=None, bit_length=8):
        super().__init__()
        self._scales = _as_t(scales)
        self._zero_point = _as_t(zero_point) if zero_point is not None else torch.zeros(1)
        self._quant_axis = -1 if quant_axis is None else quant_axis
        self._bit_length = bit_length

    def forward(self, input):
        x = _u(input)
        axis = None if self._quant_axis == -1 or self._scales.numel() == 1 else self._quant_axis
        return Tensor(Q.quantize_linear(x, self._scales.to(x.device), self._bit_length, axis)
                      .to(x.dtype))

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanter(quanter.scales(), quanter.zero_points(), quanter.quant_axis(),
                             quanter.bit_length())


class LinearDequanter(Layer):
    """q -> q * scale / range."""

    def __init__(self, scales, zero_point=None, quant_axis=None, bit_length=8):
        super().__init__()
        self._scales = _as_t(scales)
        self._zero_point = _as_t(zero_point) if zero_point is not None else torch.zeros(1)
        self._quant_axis = -1 if quant_axis is None else quant_axis
        self._bit_length = bit_length

    def forward(self, input):
        q = _u(input)
        axis = None if self._quant_axis == -1 or self._scales.numel() == 1 else self._quant_axis
        return Tensor(Q.dequantize_linear(q, self._scales.to(q.device), self._bit_length, axis)
                      .to(q.dtype))

    @staticmethod
    def from_quanter(quanter):
        return LinearDequanter(quanter.scales(), quanter.zero_points(), quanter.quant_axis(),
                               quanter.bit_length())


class LinearQuanterDequanter(Layer):
    def __init__(self, quanter, dequanter):
        super().__init__()
        self._quanter = quanter
        self._dequanter = dequanter

    def forward(self, input):
        out = input
        if self._quanter is not None:
            out = self._quanter(out)
        if self._dequanter is not None:
            out = self._dequanter(out)
        return out

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanterDequanter(LinearQuanter.from_quanter(quanter),
                                      LinearDequanter.from_quanter(quanter))


class ConvertibleQuantedLayer(Layer, metaclass=abc.ABCMeta):
    """A quanted layer that can be converted for deployment: weights are quantized in
    place (fake-quantized values stored) and activation quanters become
    quantize/dequantize pairs."""

    def __init__(self):
        super().__init__()
        self.converted = False

    @abc.abstractmethod
    def weights_to_quanters(self):
        """[(weight attribute name, quanter attribute name), ...]"""

    @abc.abstractmethod
    def activation_quanters(self):
        """[quanter attribute name, ...]"""

    def _convert_quanter_to_qdq(self, quanter_name):
        quanter = getattr(self, quanter_name)
        if quanter is None:
            return None
        qdq = LinearQuanterDequanter.from_quanter(quanter)
        setattr(self, quanter_name, qdq)
        self._sub_layers[quanter_name] = qdq
        return qdq

    def _quant_weights(self, weight_name, quanter):
        w = getattr(self, weight_name)
        with torch.no_grad():
            _u(w).copy_(_u(quanter(w)))

    def _convert(self):
        for weight_name, quanter_name in self.weights_to_quanters():
            qdq = self._convert_quanter_to_qdq(quanter_name)
            if qdq is not None:
                self._quant_weights(weight_name, qdq._quanter)
                setattr(self, quanter_name, qdq._dequanter)
                self._sub_layers[quanter_name] = qdq._dequanter
        for quanter_name in self.activation_quanters():
            self._convert_quanter_to_qdq(quanter_name)
        self.converted = True
