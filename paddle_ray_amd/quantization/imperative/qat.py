"""ImperativeQuantAware: in-place QAT rewrite of a dygraph model (parity:
python/paddle/quantization/imperative/qat.py ImperativeQuantAware / ImperativeQuantizeInputs /
ImperativeQuantizeOutputs).

quantize(model) swaps every quantizable sublayer (Conv2D, Conv2DTranspose, Linear and the
tensor-parallel linears; layers with ``skip_quant = True`` are left alone) for its
fake-quantized twin, then wraps quantized layers and activation layers in output-scale
observers. save_quantized_model() freezes the model (eval), records every observed scale
in ``<path>.quant.json`` and exports the program with ``jit.save``.
"""
import json

from ... import nn
from ...framework.core import _u
from ...nn.quant import quant_layers as QL

_QUANT_MAP = {'Conv2D': QL.QuantizedConv2D, 'Conv2DTranspose': QL.QuantizedConv2DTranspose,
              'Linear': QL.QuantizedLinear,
              'ColumnParallelLinear': QL.QuantizedColumnParallelLinear,
              'RowParallelLinear': QL.QuantizedRowParallelLinear}
_OUTPUT_OBSERVED = (nn.ReLU, nn.ReLU6, nn.LeakyReLU, nn.Sigmoid, nn.Tanh, nn.Hardswish,
                    nn.Swish, nn.Softmax, nn.AvgPool2D, nn.MaxPool2D, nn.AdaptiveAvgPool2D,
                    nn.BatchNorm2D)


def _layer_type_name(layer):
    return type(layer).__name__


class ImperativeQuantAware:
    def __init__(self, quantizable_layer_type=('Conv2D', 'Linear', 'Conv2DTranspose',
                                               'ColumnParallelLinear', 'RowParallelLinear'),
                 weight_quantize_type='abs_max',
                 activation_quantize_type='moving_average_abs_max', weight_bits=8,
                 activation_bits=8, moving_rate=0.9, fuse_conv_bn=False,
                 weight_preprocess_layer=None, act_preprocess_layer=None,
                 weight_quantize_layer=None, act_quantize_layer=None, onnx_format=False):
        names = [t if isinstance(t, str) else t.__name__ for t in quantizable_layer_type]
        for n in names:
            if n not in _QUANT_MAP:
                raise ValueError(f"{n} is not supported to be quantized")
        if activation_quantize_type not in ('moving_average_abs_max', 'abs_max'):
            raise ValueError(f"unsupported activation_quantize_type {activation_quantize_type}")
        if weight_quantize_type not in ('abs_max', 'channel_wise_abs_max'):
            raise ValueError(f"unsupported weight_quantize_type {weight_quantize_type}")
        self._types = set(names)
        self._kw = dict(weight_bits=weight_bits, activation_bits=activation_bits,
                        moving_rate=moving_rate, weight_quantize_type=weight_quantize_type,
                        activation_quantize_type=activation_quantize_type)
        self._pre = (weight_preprocess_layer, act_preprocess_layer)
        self._qlayers = (weight_quantize_layer, act_quantize_layer)
        self._fuse_conv_bn, self._onnx_format = fuse_conv_bn, onnx_format
        self._moving_rate, self._activation_bits = moving_rate, activation_bits

    def _make(self, layer):
        cls = _QUANT_MAP[_layer_type_name(layer)]
        wp, ap = self._pre
        wq, aq = self._qlayers
        return cls(layer, weight_pre_layer=wp() if wp else None,
                   act_pre_layer=ap() if ap else None,
                   weight_quant_layer=wq() if wq else None,
                   act_quant_layer=aq() if aq else None, **self._kw)

    def _quantize_inputs(self, model):
        for name, child in list(model.named_children()):
            if getattr(child, 'skip_quant', False):
                continue
            if _layer_type_name(child) in self._types:
                model._sub_layers[name] = self._make(child)
            else:
                self._quantize_inputs(child)

    def _quantize_outputs(self, model):
        for name, child in list(model.named_children()):
            if isinstance(child, (QL._QuantizedBase,)) or isinstance(child, _OUTPUT_OBSERVED):
                wrap = QL.FakeQuantMAOutputScaleLayer if self._onnx_format else \
                    QL.MAOutputScaleLayer
                if wrap is QL.FakeQuantMAOutputScaleLayer:
                    model._sub_layers[name] = wrap(child, activation_bits=self._activation_bits,
                                                   moving_rate=self._moving_rate)
                else:
                    model._sub_layers[name] = wrap(child, moving_rate=self._moving_rate)
            elif not isinstance(child, (QL.MAOutputScaleLayer, QL.FakeQuantMAOutputScaleLayer)):
                self._quantize_outputs(child)

    def quantize(self, model):
        """Rewrite ``model`` in place for quantization-aware training."""
        if self._fuse_conv_bn:
            from .fuse_utils import find_conv_bn_pairs, fuse_layers
            fuse_layers(model, find_conv_bn_pairs(model), inplace=True)
        self._quantize_inputs(model)
        self._quantize_outputs(model)
        return model

    @staticmethod
    def collect_scales(model):
        out = {}
        for name, layer in model.named_sublayers():
            for attr in ('_scale',):
                p = layer.__dict__.get('_parameters', {}).get(attr)
                if p is not None:
                    out[name] = _u(p).detach().float().cpu().reshape(-1).tolist()
        return out

    def save_quantized_model(self, layer, path, input_spec=None, **config):
        from ... import jit
        was_training = layer.training
        layer.eval()
        with open(path + '.quant.json', 'w') as f:
            json.dump({'weight_bits': self._kw['weight_bits'],
                       'activation_bits': self._kw['activation_bits'],
                       'scales': self.collect_scales(layer)}, f, indent=1)
        if input_spec is not None:
            jit.save(layer, path, input_spec=input_spec, **config)
        if was_training:
            layer.train()
