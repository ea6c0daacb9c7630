"""Built-in observers (parity: python/paddle/quantization/observers/abs_max.py)."""
import torch

from ...framework.core import Tensor, _u
from ...ops import quant as Q
from ..base import BaseObserver, ObserverFactory


class AbsmaxObserver(ObserverFactory):
    """Collects the running max |x| of the observed tensor (per-tensor)."""

    def __init__(self, quant_bits=8):
        super().__init__(quant_bits=quant_bits)

    def _get_class(self):
        return AbsmaxObserverLayer


class AbsmaxObserverLayer(BaseObserver):
    INIT_ABS_MAX = 1e-7

    def __init__(self, layer, quant_bits=8):
        super().__init__()
        self._quant_bits = quant_bits
        self.abs_max_val = Tensor(torch.tensor(self.INIT_ABS_MAX))
        self.thresholds = None

    def forward(self, input):
        x = _u(input)
        cur = Q.absmax(x)
        self.abs_max_val = Tensor(torch.maximum(cur, _u(self.abs_max_val).to(cur.device)))
        return input

    def cal_thresholds(self):
        self.thresholds = self.abs_max_val

    def bit_length(self):
        return self._quant_bits

    def quant_axis(self):
        return -1

    def scales(self):
        return self.abs_max_val

    def zero_points(self):
        return None


__all__ = ['AbsmaxObserver']
