"""QAT layers (parity: python/paddle/nn/quant/qat/{linear,conv}.py)."""
from ...functional import linear as _linear, conv2d as _conv2d
from ..format import ConvertibleQuantedLayer


class QuantedLinear(ConvertibleQuantedLayer):
    """Linear with fake-quantized input and weight (quanters from a QuantConfig entry)."""

    def __init__(self, layer, q_config):
        super().__init__()
        self.weight, self.bias = layer.weight, layer.bias
        self.name = getattr(layer, 'name', None)
        self.weight_quanter = q_config.weight._instance(layer) if q_config.weight is not None \
            else None
        self.activation_quanter = q_config.activation._instance(layer) \
            if q_config.activation is not None else None

    def forward(self, input):
        x = self.activation_quanter(input) if self.activation_quanter is not None else input
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        return _linear(x, w, self.bias)

    def weights_to_quanters(self):
        return [('weight', 'weight_quanter')]

    def activation_quanters(self):
        return ['activation_quanter']


class QuantedConv2D(ConvertibleQuantedLayer):
    def __init__(self, layer, q_config):
        super().__init__()
        self.weight, self.bias = layer.weight, layer.bias
        self._stride, self._padding = layer._stride, layer._padding
        self._dilation, self._groups = layer._dilation, layer._groups
        self._data_format = layer._data_format
        self.weight_quanter = q_config.weight._instance(layer) if q_config.weight is not None \
            else None
        self.activation_quanter = q_config.activation._instance(layer) \
            if q_config.activation is not None else None

    def forward(self, input):
        x = self.activation_quanter(input) if self.activation_quanter is not None else input
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        return _conv2d(x, w, self.bias, self._stride, self._padding, self._dilation, self._groups,
                       self._data_format)

    def weights_to_quanters(self):
        return [('weight', 'weight_quanter')]

    def activation_quanters(self):
        return ['activation_quanter']


__all__ = ['QuantedLinear', 'QuantedConv2D']
