"""Quantization stubs (parity: python/paddle/nn/quant/stub.py)."""
from ..layer.layers import Layer


class Stub(Layer):
    """Identity placeholder that QAT/PTQ replace with an observer of its input."""

    def __init__(self, observer=None):
        super().__init__()
        self._observer = observer

    def forward(self, input):
        return input


class QuanterStub(Layer):
    """Identity with an observer (created from the stub's factory or the layer config)."""

    def __init__(self, layer, q_config):
        super().__init__()
        self._observer = None
        if layer._observer is not None:
            self._observer = layer._observer._instance(layer)
        elif q_config.activation is not None:
            self._observer = q_config.activation._instance(layer)

    def forward(self, input):
        return self._observer(input) if self._observer is not None else input
