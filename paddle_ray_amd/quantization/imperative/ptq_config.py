"""PTQConfig (parity: python/paddle/quantization/imperative/ptq_config.py)."""
import copy

from .ptq_quantizer import (AbsmaxQuantizer, BaseQuantizer, PerChannelAbsmaxQuantizer,
                            SUPPORT_ACT_QUANTIZERS, SUPPORT_WT_QUANTIZERS)


class PTQConfig:
    def __init__(self, activation_quantizer, weight_quantizer):
        if type(activation_quantizer) not in SUPPORT_ACT_QUANTIZERS:
            raise TypeError("The activation quantizer is not supported")
        if type(weight_quantizer) not in SUPPORT_WT_QUANTIZERS:
            raise TypeError("The weight quantizer is not supported")
        self.in_act_quantizer = copy.deepcopy(activation_quantizer)
        self.out_act_quantizer = copy.deepcopy(activation_quantizer)
        self.wt_quantizer = copy.deepcopy(weight_quantizer)
        self.quant_hook_handle = None
        self.enable_in_act_quantizer = False


default_ptq_config = PTQConfig(AbsmaxQuantizer(), AbsmaxQuantizer())
__all__ = ['PTQConfig', 'default_ptq_config', 'BaseQuantizer', 'PerChannelAbsmaxQuantizer']
