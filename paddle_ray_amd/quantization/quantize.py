"""QAT / PTQ drivers (parity: python/paddle/quantization/{quantize,qat,ptq}.py)."""
import abc
import copy

from .base import BaseQuanter
from .config import QuantConfig


class Quantization(metaclass=abc.ABCMeta):
    def __init__(self, config: QuantConfig):
        self._config = copy.deepcopy(config)

    @abc.abstractmethod
    def quantize(self, model, inplace=False):
        ...

    def convert(self, model, inplace=False):
        """Deployment form: quanted layers quantize their weights in place and activation
        quanters become LinearQuanter/LinearDequanter pairs."""
        from ..nn.quant.format import ConvertibleQuantedLayer, LinearQuanterDequanter
        m = model if inplace else copy.deepcopy(model)
        replaced = {}
        for name, child in m.named_children():
            if isinstance(child, ConvertibleQuantedLayer):
                child._convert()
            elif isinstance(child, BaseQuanter):
                replaced[name] = LinearQuanterDequanter.from_quanter(child)
            else:
                self.convert(child, inplace=True)
        for k, v in replaced.items():
            m._sub_layers[k] = v
        return m

    def _convert_to_quant_layers(self, model, config):
        replaced = {}
        for name, child in model.named_children():
            if config._is_quantifiable(child) and type(child) in config.qat_layer_mappings:
                replaced[name] = config._get_qat_layer(child)
            else:
                self._convert_to_quant_layers(child, config)
        for k, v in replaced.items():
            model._sub_layers[k] = v

    def _insert_activation_observers(self, model, config):
        replaced = {}
        for name, child in model.named_children():
            if config._need_observe(child):
                replaced[name] = config._get_observe_wrapper(child)
            else:
                self._insert_activation_observers(child, config)
        for k, v in replaced.items():
            model._sub_layers[k] = v

    def _details(self):
        return self._config.details()

    def __str__(self):
        return self._details()

    __repr__ = __str__


class QAT(Quantization):
    """Quantization-aware training: quanted layers + fake quanters on activations."""

    def quantize(self, model, inplace=False):
        if not model.training:
            raise RuntimeError("Quantization-Aware Training shoud work on training models. "
                               "Please set training mode by model.train().")
        m = model if inplace else copy.deepcopy(model)
        self._config._specify(m)
        self._convert_to_quant_layers(m, self._config)
        self._insert_activation_observers(m, self._config)
        return m


class PTQ(Quantization):
    """Post-training quantization: observers collect ranges during calibration runs."""

    def quantize(self, model, inplace=False):
        m = model
        if not inplace:
            m = copy.deepcopy(model)
            m.eval()
        if model.training and inplace:
            raise RuntimeError("Post-Training Quantization shoud not work on training models. "
                               "Please set evaluation mode by model.eval().")
        self._config._specify(m)
        self._convert_to_quant_layers(m, self._config)
        self._insert_activation_observers(m, self._config)
        return m
