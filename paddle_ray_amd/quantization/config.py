"""QuantConfig (parity: python/paddle/quantization/config.py): per-layer quantization
configuration resolved with priority layer > full name > type > parent > global."""
import copy

from .. import nn
from ..nn.layer.layers import Layer
from .base import ObserveWrapper


def _default_qat_mappings():
    from ..nn.quant import qat, stub
    return {stub.Stub: stub.QuanterStub, nn.Linear: qat.QuantedLinear,
            nn.Conv2D: qat.QuantedConv2D}


DEFAULT_LEAVES = [nn.ReLU, nn.AvgPool2D]


class SingleLayerConfig:
    def __init__(self, activation, weight):
        self._activation, self._weight = activation, weight

    @property
    def activation(self):
        return self._activation

    @property
    def weight(self):
        return self._weight

    def __str__(self):
        return f"activation: {self._activation}\nweight: {self._weight}"


class QuantConfig:
    def __init__(self, activation, weight):
        self._global_config = None if (activation is None and weight is None) else \
            SingleLayerConfig(activation, weight)
        self._layer2config = {}
        self._prefix2config = {}
        self._type2config = {}
        self._model = None
        self._qat_layer_mapping = dict(_default_qat_mappings())
        self._customized_qat_layer_mapping = {}
        self._customized_leaves = []

    # -- configuration -------------------------------------------------------------
    def add_layer_config(self, layer, activation=None, weight=None):
        if isinstance(layer, list):
            for l in layer:
                self.add_layer_config(l, activation, weight)
        else:
            self.add_name_config(layer.full_name(), activation, weight)

    def add_name_config(self, layer_name, activation=None, weight=None):
        if isinstance(layer_name, str):
            self._prefix2config[layer_name] = SingleLayerConfig(activation, weight)
        elif isinstance(layer_name, list):
            for n in layer_name:
                self.add_name_config(n, activation, weight)

    def add_type_config(self, layer_type, activation=None, weight=None):
        if isinstance(layer_type, type) and issubclass(layer_type, Layer):
            self._type2config[layer_type] = SingleLayerConfig(activation, weight)
        elif isinstance(layer_type, list):
            for t in layer_type:
                self.add_type_config(t, activation, weight)

    def add_qat_layer_mapping(self, source, target):
        if not (isinstance(source, type) and issubclass(source, Layer)):
            raise TypeError("The source layer to be placed should be a subclass of paddle.nn.Layer")
        if not isinstance(target, type):
            raise TypeError("The target layer should be a class")
        self._qat_layer_mapping[source] = target
        self._customized_qat_layer_mapping[source] = target

    def add_customized_leaf(self, layer_type):
        self._customized_leaves.append(layer_type)

    @property
    def customized_leaves(self):
        return self._customized_leaves

    @property
    def qat_layer_mappings(self):
        return self._qat_layer_mapping

    @property
    def default_qat_layer_mapping(self):
        return _default_qat_mappings()

    @property
    def global_config(self):
        return self._global_config

    # -- resolution ------------------------------------------------------------------
    def _get_config_by_layer(self, layer):
        return self._layer2config.get(layer, None)

    def _is_quantifiable(self, layer):
        return layer in self._layer2config

    def _need_observe(self, layer):
        return self._is_leaf(layer) and self._has_observer_config(layer)

    def _has_observer_config(self, layer):
        c = self._get_config_by_layer(layer)
        return c is not None and c.activation is not None

    def _is_leaf(self, layer):
        return (type(layer) in DEFAULT_LEAVES or len(layer._sub_layers) == 0 or
                type(layer) in self._customized_leaves)

    def _get_qat_layer(self, layer):
        cfg = self._get_config_by_layer(layer)
        target = self._customized_qat_layer_mapping.get(type(layer),
                                                        self._qat_layer_mapping.get(type(layer)))
        return target(layer, cfg)

    def _get_observer(self, layer):
        c = self._get_config_by_layer(layer)
        obs = None if c is None else c.activation
        return None if obs is None else obs._instance(layer)

    def _get_observe_wrapper(self, layer):
        return ObserveWrapper(self._get_observer(layer), layer)

    def _specify(self, model):
        self._model = model
        self._specify_helper(model)

    def _specify_helper(self, model):
        for child in model.children():
            cfg = self._layer2config.get(model, self._global_config)
            cfg = self._type2config.get(type(child), cfg)
            cfg = self._prefix2config.get(child.full_name(), cfg)
            if cfg is not None:
                self._layer2config[child] = cfg
            self._specify_helper(child)
        return self

    def details(self):
        if self._model is None:
            return str(self)
        return self._details_helper(self._model)

    def _details_helper(self, layer, indent=0):
        lines = []
        for name, sub in layer.named_children():
            s = self._details_helper(sub, indent + 2)
            if sub in self._layer2config:
                lines.append(f"({name}): {s}, {self._layer2config[sub]}")
        out = layer.__class__.__name__ + '('
        if lines:
            out += '\n  ' + '\n  '.join(lines) + '\n'
        return out + ')'

    def __str__(self):
        parts = [f"Global config:\n{self._global_config}"]
        if self._type2config:
            parts.append("Layer type config:\n" + str(self._type2config))
        if self._prefix2config:
            parts.append("Layer prefix config:\n" + str(self._prefix2config))
        return "\n".join(parts)

    def __deepcopy__(self, memo):
        new = copy.copy(self)
        new._layer2config = dict(self._layer2config)
        new._prefix2config = dict(self._prefix2config)
        new._type2config = dict(self._type2config)
        new._qat_layer_mapping = dict(self._qat_layer_mapping)
        new._customized_qat_layer_mapping = dict(self._customized_qat_layer_mapping)
        new._customized_leaves = list(self._customized_leaves)
        return new
