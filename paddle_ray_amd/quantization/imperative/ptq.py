"""ImperativePTQ: calibration-based post-training quantization of a dygraph model (parity:
python/paddle/quantization/imperative/ptq.py).

quantize() attaches a PTQConfig copy to every supported sublayer plus a forward-post hook
that feeds the layer's input / output activations to the activation quantizer and, once,
the weight to the weight quantizer. Run calibration batches, then save_quantized_model()
(or convert()) computes the thresholds, drops the hooks, replaces Conv2D/Linear with
fake-quantized layers whose scales are the calibrated thresholds, and exports.
"""
import copy
import json

import torch

from ...framework.core import _u
from ...nn.quant import quant_layers as QL
from .ptq_config import default_ptq_config
from .ptq_registry import PTQRegistry


class ImperativePTQ:
    def __init__(self, quant_config=default_ptq_config):
        self._quant_config = quant_config

    @staticmethod
    def _is_leaf(layer):
        return not list(layer.children())

    def quantize(self, model, inplace=False, fuse=False, fuse_list=None):
        m = model if inplace else copy.deepcopy(model)
        if fuse:
            from .fuse_utils import find_conv_bn_pairs, fuse_layers
            fuse_layers(m, fuse_list or find_conv_bn_pairs(m), inplace=True)
        for _, layer in m.named_sublayers():
            if PTQRegistry.is_supported_layer(layer) and self._is_leaf(layer):
                cfg = copy.deepcopy(self._quant_config)
                if PTQRegistry.is_simulated_quant_layer(layer):
                    cfg.enable_in_act_quantizer = True
                layer._quant_config = cfg
                cfg.quant_hook_handle = layer.register_forward_post_hook(self._hook)
        return m

    @staticmethod
    def _hook(layer, inputs, outputs):
        cfg = layer._quant_config
        if layer.training:
            return None
        ins = [i for i in (inputs if isinstance(inputs, (list, tuple)) else [inputs])
               if hasattr(i, 'shape')]
        outs = [o for o in (outputs if isinstance(outputs, (list, tuple)) else [outputs])
                if hasattr(o, 'shape')]
        if cfg.enable_in_act_quantizer:
            cfg.in_act_quantizer.sample_data(layer, ins)
        cfg.out_act_quantizer.sample_data(layer, outs)
        if getattr(layer, 'weight', None) is not None and not cfg.wt_quantizer.abs_max_vals:
            cfg.wt_quantizer.sample_data(layer, [layer.weight])
        return None

    def _cal_thresholds(self, model):
        info = {}
        for name, layer in model.named_sublayers():
            cfg = getattr(layer, '_quant_config', None)
            if cfg is None:
                continue
            if cfg.enable_in_act_quantizer:
                cfg.in_act_quantizer.cal_thresholds()
            cfg.out_act_quantizer.cal_thresholds()
            if cfg.wt_quantizer.abs_max_vals:
                cfg.wt_quantizer.cal_thresholds()
            if cfg.quant_hook_handle is not None:
                cfg.quant_hook_handle.remove()
                cfg.quant_hook_handle = None
            info[name] = {
                'in_threshold': list(map(float, cfg.in_act_quantizer.thresholds))
                if cfg.enable_in_act_quantizer else [],
                'out_threshold': list(map(float, cfg.out_act_quantizer.thresholds)),
                'weight_threshold': [list(map(float, t)) if isinstance(t, (list, tuple)) else
                                     float(t) for t in cfg.wt_quantizer.thresholds]}
        return info

    @staticmethod
    def _simulated(layer, cfg):
        """Conv2D/Linear -> fake-quantized twin with frozen calibrated scales."""
        wq = cfg.wt_quantizer
        per_channel = wq.thresholds and isinstance(wq.thresholds[0], (list, tuple))
        cls = QL.QuantizedLinear if type(layer).__name__ == 'Linear' else QL.QuantizedConv2D
        q = cls(layer, weight_bits=wq.quant_bits, activation_bits=cfg.in_act_quantizer.quant_bits,
                weight_quantize_type='channel_wise_abs_max' if per_channel else 'abs_max',
                activation_quantize_type='moving_average_abs_max')
        if cfg.in_act_quantizer.thresholds:
            with torch.no_grad():
                _u(q._fake_quant_input._scale).fill_(float(cfg.in_act_quantizer.thresholds[0]))
        return q

    def convert(self, model, inplace=True):
        m = model if inplace else copy.deepcopy(model)
        info = self._cal_thresholds(m)
        self._wrap(m)
        m.eval()
        m._ptq_thresholds = info
        return m

    def _wrap(self, model):
        for name, child in list(model.named_children()):
            cfg = getattr(child, '_quant_config', None)
            if cfg is not None and PTQRegistry.is_simulated_quant_layer(child):
                model._sub_layers[name] = self._simulated(child, cfg)
            else:
                self._wrap(child)

    def save_quantized_model(self, model, path, input_spec=None, **config):
        m = self.convert(model, inplace=True)
        with open(path + '.quant.json', 'w') as f:
            json.dump(m._ptq_thresholds, f, indent=1)
        if input_spec is not None:
            from ... import jit
            jit.save(m, path, input_spec=input_spec, **config)
        return m
