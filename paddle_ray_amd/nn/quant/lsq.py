"""Learned step-size quantization (LSQ / LSQ+) fake quanters (parity:
python/paddle/nn/quant/lsq.py): the step size (and LSQ+ offset) are trainable, with the
LSQ gradient scale g = 1 / sqrt(N * Qp)."""
import math

import torch

from ...framework.core import Tensor, _u
from .. import initializer as I
from ..layer.layers import Layer, ParamAttr


def _round_ste(x):
    return (x.round() - x).detach() + x


def _grad_scale(x, scale):
    return (x - x * scale).detach() + x * scale


class FakeQuantActLSQPlus(Layer):
    def __init__(self, quant_bits, all_postive=False, symmetric=False, batch_init=20,
                 dtype='float32', name=None, reduce_type=None):
        super().__init__()
        self.bits, self.all_positive, self.symmetric = quant_bits, all_postive, symmetric
        self.batch_init, self.reduce_type = batch_init, reduce_type
        if all_postive:
            self.Qn, self.Qp = 0, 2 ** quant_bits - 1
        else:
            self.Qn, self.Qp = -2 ** (quant_bits - 1), 2 ** (quant_bits - 1) - 1
        self.s = self.create_parameter([1], ParamAttr(initializer=I.Constant(1.0)), dtype=dtype)
        self.beta = self.create_parameter([1], ParamAttr(initializer=I.Constant(0.0)),
                                          dtype=dtype)
        self.init_state = 0

    def forward(self, activation):
        x = _u(activation)
        s, beta = _u(self.s), _u(self.beta)
        if self.init_state < self.batch_init and self.training:
            with torch.no_grad():
                if self.symmetric:
                    s.copy_((x.abs().max() / max(self.Qp, 1)).reshape(1).clamp_min(1e-8))
                else:
                    mn, mx = x.min(), x.max()
                    s.copy_(((mx - mn) / (self.Qp - self.Qn)).reshape(1).clamp_min(1e-8))
                    beta.copy_((mn - s[0] * self.Qn).reshape(1))
            self.init_state += 1
        g = 1.0 / math.sqrt(x.numel() * max(self.Qp, 1))
        ss = _grad_scale(s, g)
        bb = _grad_scale(beta, g) if not self.symmetric else torch.zeros_like(beta)
        q = torch.clamp(_round_ste((x - bb) / ss), self.Qn, self.Qp)
        return Tensor(q * ss + bb)


class FakeQuantWeightLSQPlus(Layer):
    def __init__(self, quant_bits, all_postive=False, per_channel=False, batch_init=20,
                 channel_num=None, quant_linear=False, dtype='float32', name=None,
                 reduce_type=None):
        super().__init__()
        self.bits, self.per_channel, self.batch_init = quant_bits, per_channel, batch_init
        self.quant_linear, self.reduce_type = quant_linear, reduce_type
        self.Qn, self.Qp = (0, 2 ** quant_bits - 1) if all_postive else \
            (-2 ** (quant_bits - 1), 2 ** (quant_bits - 1) - 1)
        n = channel_num if per_channel else 1
        self.s = self.create_parameter([n], ParamAttr(initializer=I.Constant(1.0)), dtype=dtype)
        self.init_state = 0

    def forward(self, weight):
        w = _u(weight)
        s = _u(self.s)
        axis = (w.dim() - 1) if self.quant_linear else 0
        if self.init_state < self.batch_init:
            with torch.no_grad():
                if self.per_channel:
                    dims = [d for d in range(w.dim()) if d != axis]
                    mean, std = w.mean(dims), w.std(dims)
                    s.copy_(torch.maximum((mean - 3 * std).abs(), (mean + 3 * std).abs())
                            / 2 ** (self.bits - 1))
                else:
                    mean, std = w.mean(), w.std()
                    s.copy_((torch.maximum((mean - 3 * std).abs(), (mean + 3 * std).abs())
                             / 2 ** (self.bits - 1)).reshape(1))
                s.clamp_(min=1e-8)
            self.init_state += 1
        g = 1.0 / math.sqrt(w.numel() * max(self.Qp, 1))
        ss = _grad_scale(s, g)
        if self.per_channel:
            shape = [1] * w.dim()
            shape[axis] = -1
            ss = ss.reshape(shape)
        q = torch.clamp(_round_ste(w / ss), self.Qn, self.Qp)
        return Tensor(q * ss)
