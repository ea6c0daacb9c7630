"""Parameter initializers (parity: python/paddle/nn/initializer/*).

Initialisation runs on the parameter's own device (HBM) with torch's Philox
generator — no host round trip for 1B+ parameter models.
"""
import math

import numpy as np
import torch

from ...framework.core import Tensor, _u

_global_weight_init = [None]
_global_bias_init = [None]


def _fans(shape):
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        # paddle Linear weight is [in, out]
        return shape[0], shape[1]
    rf = int(np.prod(shape[2:]))
    # conv weight [out, in/groups, kh, kw]
    return shape[1] * rf, shape[0] * rf


def calculate_gain(nonlinearity, param=None):
    nl = nonlinearity.lower()
    if nl in ('sigmoid', 'linear', 'conv1d', 'conv2d', 'conv3d', 'conv1d_transpose',
              'conv2d_transpose', 'conv3d_transpose'):
        return 1.0
    if nl == 'tanh':
        return 5.0 / 3
    if nl == 'relu':
        return math.sqrt(2.0)
    if nl == 'leaky_relu':
        p = 0.01 if param is None else param
        return math.sqrt(2.0 / (1 + p ** 2))
    if nl == 'selu':
        return 3.0 / 4
    raise ValueError(f"unsupported nonlinearity {nonlinearity}")


class Initializer:
    def __call__(self, param, block=None):
        t = _u(param)
        with torch.no_grad():
            self._init(t)
        return param

    def _init(self, t):
        raise NotImplementedError


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def _init(self, t):
        t.fill_(self.value)


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, seed=0, name=None):
        self.low, self.high = low, high

    def _init(self, t):
        t.uniform_(self.low, self.high)


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, seed=0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        t.normal_(self.mean, self.std)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, seed=0, a=-2.0, b=2.0, name=None):
        self.mean, self.std, self.a, self.b = mean, std, a, b

    def _init(self, t):
        torch.nn.init.trunc_normal_(t, self.mean, self.std, self.mean + self.a * self.std,
                                    self.mean + self.b * self.std)


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        lim = self.gain * math.sqrt(6.0 / (fi + fo))
        t.uniform_(-lim, lim)


class XavierNormal(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        t.normal_(0, self.gain * math.sqrt(2.0 / (fi + fo)))


class KaimingUniform(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity='relu', name=None):
        self.fan_in, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fan_in or _fans(list(t.shape))[0]
        gain = calculate_gain(self.nl, self.slope)
        lim = gain * math.sqrt(3.0 / fi)
        t.uniform_(-lim, lim)


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity='relu', name=None):
        self.fan_in, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fan_in or _fans(list(t.shape))[0]
        gain = calculate_gain(self.nl, self.slope)
        t.normal_(0, gain / math.sqrt(fi))


MSRAInitializer = KaimingNormal


class Assign(Initializer):
    def __init__(self, value, name=None):
        self.value = value

    def _init(self, t):
        v = _u(self.value) if isinstance(self.value, Tensor) else torch.as_tensor(
            np.asarray(self.value))
        t.copy_(v.reshape(t.shape).to(t.dtype))


NumpyArrayInitializer = Assign


class Orthogonal(Initializer):
    def __init__(self, gain=1.0, name=None):
        self.gain = gain

    def _init(self, t):
        torch.nn.init.orthogonal_(t, self.gain)


class Dirac(Initializer):
    def __init__(self, groups=1, name=None):
        self.groups = groups

    def _init(self, t):
        torch.nn.init.dirac_(t, self.groups)


class Bilinear(Initializer):
    def _init(self, t):
        shape = t.shape
        f = math.ceil(shape[3] / 2)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = torch.zeros(shape[2], shape[3])
        for i in range(shape[2]):
            for j in range(shape[3]):
                w[i, j] = (1 - abs(i / f - c)) * (1 - abs(j / f - c))
        t.copy_(w.expand(shape).to(t.dtype))


def set_global_initializer(weight_init, bias_init=None):
    _global_weight_init[0] = weight_init
    _global_bias_init[0] = bias_init


def _init_param(p, attr=None, default_initializer=None, is_bias=False):
    init = None
    if attr is not None and getattr(attr, 'initializer', None) is not None:
        init = attr.initializer
    elif is_bias and _global_bias_init[0] is not None:
        init = _global_bias_init[0]
    elif not is_bias and _global_weight_init[0] is not None:
        init = _global_weight_init[0]
    elif default_initializer is not None:
        init = default_initializer
    elif is_bias:
        init = Constant(0.0)
    else:
        init = XavierUniform()
    init(p)
    return p
