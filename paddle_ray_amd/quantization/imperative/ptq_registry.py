"""Which layers PTQ can quantize and which of their inputs/outputs it observes (parity:
python/paddle/quantization/imperative/ptq_registry.py)."""
from ... import nn


class LayerInfo:
    def __init__(self, layer, input_names, weight_names, output_names):
        self.layer, self.input_names = layer, input_names
        self.weight_names, self.output_names = weight_names, output_names


PTQ_LAYERS_INFO = [
    LayerInfo(nn.Conv2D, ['Input'], ['Filter'], ['Output']),
    LayerInfo(nn.Linear, ['X'], ['Y'], ['Out']),
    LayerInfo(nn.BatchNorm2D, ['X'], [], ['Y']),
    LayerInfo(nn.AdaptiveMaxPool2D, ['X'], [], ['Out']),
    LayerInfo(nn.AdaptiveAvgPool2D, ['X'], [], ['Out']),
    LayerInfo(nn.AvgPool2D, ['X'], [], ['Out']),
    LayerInfo(nn.MaxPool2D, ['X'], [], ['Out']),
    LayerInfo(nn.ReLU, ['X'], [], ['Out']),
    LayerInfo(nn.ReLU6, ['X'], [], ['Out']),
    LayerInfo(nn.Hardswish, ['X'], [], ['Out']),
    LayerInfo(nn.Swish, ['X'], [], ['Out']),
    LayerInfo(nn.Sigmoid, ['X'], [], ['Out']),
    LayerInfo(nn.Softmax, ['X'], [], ['Out']),
    LayerInfo(nn.Tanh, ['X'], [], ['Out']),
]
QUANT_LAYERS_INFO = [LayerInfo(nn.Conv2D, ['Input'], ['Filter'], ['Output']),
                     LayerInfo(nn.Linear, ['X'], ['Y'], ['Out'])]
SIMULATED_LAYERS = [nn.Conv2D, nn.Linear]


class PTQRegistry:
    supported_layers_map = {i.layer: i for i in PTQ_LAYERS_INFO}
    registered_layers_map = {i.layer: i for i in QUANT_LAYERS_INFO}

    @classmethod
    def is_supported_layer(cls, layer):
        return layer in cls.supported_layers_map or isinstance(layer, tuple(
            cls.supported_layers_map))

    @classmethod
    def is_registered_layer(cls, layer):
        return layer in cls.registered_layers_map or isinstance(layer, tuple(
            cls.registered_layers_map))

    @classmethod
    def is_simulated_quant_layer(cls, layer):
        return layer in SIMULATED_LAYERS or isinstance(layer, tuple(SIMULATED_LAYERS))

    @classmethod
    def layer_info(cls, layer):
        for k, v in cls.supported_layers_map.items():
            if isinstance(layer, k):
                return v
        return None
