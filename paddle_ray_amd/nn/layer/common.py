"""Common layers, activations, containers (parity: python/paddle/nn/layer/{common,activation,container}.py)."""
import collections

import numpy as np
import torch

from ...framework.core import Tensor, Parameter, _u
from .. import functional as F
from .. import initializer as I
from .layers import Layer, ParamAttr


class Identity(Layer):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, x):
        return x


class Linear(Layer):
    """y = xW + b, W: [in_features, out_features] (paddle layout)."""

    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self._in_features, self._out_features = in_features, out_features
        self.weight = self.create_parameter([in_features, out_features], weight_attr)
        self.bias = self.create_parameter([out_features], bias_attr, is_bias=True)

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f'in_features={self._in_features}, out_features={self._out_features}, dtype={self._dtype}'


class Bilinear(Layer):
    def __init__(self, in1_features, in2_features, out_features, weight_attr=None, bias_attr=None,
                 name=None):
        super().__init__()
        self.weight = self.create_parameter([out_features, in1_features, in2_features], weight_attr)
        self.bias = self.create_parameter([1, out_features], bias_attr, is_bias=True)

    def forward(self, x1, x2):
        return F.bilinear(x1, x2, self.weight, self.bias)


class Embedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, sparse=False,
                 weight_attr=None, name=None):
        super().__init__()
        self._num_embeddings, self._embedding_dim = num_embeddings, embedding_dim
        if padding_idx is not None and padding_idx < 0:
            padding_idx += num_embeddings
        self._padding_idx = padding_idx
        self.weight = self.create_parameter([num_embeddings, embedding_dim], weight_attr)
        if padding_idx is not None:
            with torch.no_grad():
                self.weight._t[padding_idx] = 0

    def forward(self, x):
        return F.embedding(x, self.weight, self._padding_idx)

    def extra_repr(self):
        return f'{self._num_embeddings}, {self._embedding_dim}'


class Dropout(Layer):
    def __init__(self, p=0.5, axis=None, mode='upscale_in_train', name=None):
        super().__init__()
        self.p, self.axis, self.mode = p, axis, mode

    def forward(self, x):
        return F.dropout(x, self.p, self.axis, self.training, self.mode)

    def extra_repr(self):
        return f'p={self.p}, axis={self.axis}, mode={self.mode}'


class Dropout2D(Layer):
    def __init__(self, p=0.5, data_format='NCHW', name=None):
        super().__init__()
        self.p, self.data_format = p, data_format

    def forward(self, x):
        return F.dropout2d(x, self.p, self.training, self.data_format)


class Dropout3D(Layer):
    def __init__(self, p=0.5, data_format='NCDHW', name=None):
        super().__init__()
        self.p = p

    def forward(self, x):
        return F.dropout3d(x, self.p, self.training)


class AlphaDropout(Layer):
    def __init__(self, p=0.5, name=None):
        super().__init__()
        self.p = p

    def forward(self, x):
        return F.alpha_dropout(x, self.p, self.training)


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self.start_axis, self.stop_axis = start_axis, stop_axis

    def forward(self, x):
        return Tensor(_u(x).flatten(self.start_axis, self.stop_axis))


class Unflatten(Layer):
    def __init__(self, axis, shape, name=None):
        super().__init__()
        self.axis, self.shape = axis, shape

    def forward(self, x):
        return Tensor(_u(x).unflatten(self.axis, list(self.shape)))


class Upsample(Layer):
    def __init__(self, size=None, scale_factor=None, mode='nearest', align_corners=False,
                 align_mode=0, data_format='NCHW', name=None):
        super().__init__()
        self.size, self.scale_factor, self.mode = size, scale_factor, mode
        self.align_corners, self.data_format = align_corners, data_format

    def forward(self, x):
        return F.interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners,
                             data_format=self.data_format)


class UpsamplingNearest2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format='NCHW', name=None):
        super().__init__(size, scale_factor, 'nearest', data_format=data_format)


class UpsamplingBilinear2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format='NCHW', name=None):
        super().__init__(size, scale_factor, 'bilinear', True, data_format=data_format)


class _PadN(Layer):
    def __init__(self, padding, mode='constant', value=0.0, data_format='NCHW', name=None, n=2):
        super().__init__()
        if isinstance(padding, int):
            padding = [padding] * (2 * n)
        self.padding, self.mode, self.value, self.data_format = padding, mode, value, data_format

    def forward(self, x):
        return F.pad(x, self.padding, self.mode, self.value, self.data_format)


class Pad1D(_PadN):
    def __init__(self, padding, mode='constant', value=0.0, data_format='NCL', name=None):
        super().__init__(padding, mode, value, data_format, name, 1)


class Pad2D(_PadN):
    def __init__(self, padding, mode='constant', value=0.0, data_format='NCHW', name=None):
        super().__init__(padding, mode, value, data_format, name, 2)


class Pad3D(_PadN):
    def __init__(self, padding, mode='constant', value=0.0, data_format='NCDHW', name=None):
        super().__init__(padding, mode, value, data_format, name, 3)


class ZeroPad2D(Pad2D):
    def __init__(self, padding, data_format='NCHW', name=None):
        super().__init__(padding, 'constant', 0.0, data_format)


class CosineSimilarity(Layer):
    def __init__(self, axis=1, eps=1e-8):
        super().__init__()
        self.axis, self.eps = axis, eps

    def forward(self, x1, x2):
        return F.cosine_similarity(x1, x2, self.axis, self.eps)


class PairwiseDistance(Layer):
    def __init__(self, p=2., epsilon=1e-6, keepdim=False, name=None):
        super().__init__()
        self.p, self.epsilon, self.keepdim = p, epsilon, keepdim

    def forward(self, x, y):
        return F.pairwise_distance(x, y, self.p, self.epsilon, self.keepdim)


class Unfold(Layer):
    def __init__(self, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.args = (kernel_sizes, strides, paddings, dilations)

    def forward(self, x):
        return F.unfold(x, *self.args)


class Fold(Layer):
    def __init__(self, output_sizes, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.args = (output_sizes, kernel_sizes, strides, paddings, dilations)

    def forward(self, x):
        return F.fold(x, *self.args)


class PixelShuffle(Layer):
    def __init__(self, upscale_factor, data_format='NCHW', name=None):
        super().__init__()
        self.f, self.df = upscale_factor, data_format

    def forward(self, x):
        return F.pixel_shuffle(x, self.f, self.df)


class PixelUnshuffle(Layer):
    def __init__(self, downscale_factor, data_format='NCHW', name=None):
        super().__init__()
        self.f, self.df = downscale_factor, data_format

    def forward(self, x):
        return F.pixel_unshuffle(x, self.f, self.df)


class ChannelShuffle(Layer):
    def __init__(self, groups, data_format='NCHW', name=None):
        super().__init__()
        self.g, self.df = groups, data_format

    def forward(self, x):
        return F.channel_shuffle(x, self.g, self.df)


# -- activations -------------------------------------------------------------------
def _act(name, fn, **defaults):
    def __init__(self, *args, name=None, **kwargs):
        Layer.__init__(self)
        params = dict(defaults)
        for k, a in zip(list(defaults), args):
            params[k] = a
        params.update({k: v for k, v in kwargs.items() if k in defaults})
        self._params = params

    def forward(self, x):
        return fn(x, **self._params)

    def extra_repr(self):
        return ', '.join(f'{k}={v}' for k, v in self._params.items())

    return type(name, (Layer,), {'__init__': __init__, 'forward': forward, 'extra_repr': extra_repr})


ReLU = _act('ReLU', F.relu)
ReLU6 = _act('ReLU6', F.relu6)
LeakyReLU = _act('LeakyReLU', F.leaky_relu, negative_slope=0.01)
ELU = _act('ELU', F.elu, alpha=1.0)
CELU = _act('CELU', F.celu, alpha=1.0)
SELU = _act('SELU', F.selu, scale=1.0507009873554804934193349852946,
            alpha=1.6732632423543772848170429916717)
GELU = _act('GELU', F.gelu, approximate=False)
Silu = _act('Silu', F.silu)
Swish = _act('Swish', F.swish)
Mish = _act('Mish', F.mish)
Sigmoid = _act('Sigmoid', F.sigmoid)
Tanh = _act('Tanh', F.tanh)
Hardtanh = _act('Hardtanh', F.hardtanh, min=-1.0, max=1.0)
Hardsigmoid = _act('Hardsigmoid', F.hardsigmoid)
Hardswish = _act('Hardswish', F.hardswish)
Hardshrink = _act('Hardshrink', F.hardshrink, threshold=0.5)
Softshrink = _act('Softshrink', F.softshrink, threshold=0.5)
Softsign = _act('Softsign', F.softsign)
Softplus = _act('Softplus', F.softplus, beta=1, threshold=20)
Tanhshrink = _act('Tanhshrink', F.tanhshrink)
ThresholdedReLU = _act('ThresholdedReLU', F.thresholded_relu, threshold=1.0)
LogSigmoid = _act('LogSigmoid', F.log_sigmoid)
Softmax = _act('Softmax', F.softmax, axis=-1)
LogSoftmax = _act('LogSoftmax', F.log_softmax, axis=-1)
Maxout = _act('Maxout', F.maxout, groups=2, axis=1)
GLU = _act('GLU', F.glu, axis=-1)
RReLU = _act('RReLU', F.rrelu, lower=1. / 8., upper=1. / 3.)


class Softmax2D(Layer):
    def forward(self, x):
        return F.softmax(x, axis=-3)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format='NCHW', name=None):
        super().__init__()
        self._data_format = data_format
        self.weight = self.create_parameter([num_parameters], weight_attr,
                                            default_initializer=I.Constant(init))

    def forward(self, x):
        return F.prelu(x, self.weight, self._data_format)


# -- containers ----------------------------------------------------------------------
class Sequential(Layer):
    def __init__(self, *layers):
        super().__init__()
        if len(layers) == 1 and isinstance(layers[0], (list, tuple)) and layers[0] and \
                isinstance(layers[0][0], (list, tuple)):
            for n, l in layers[0]:
                self.add_sublayer(n, l)
        elif len(layers) == 1 and isinstance(layers[0], collections.OrderedDict):
            for n, l in layers[0].items():
                self.add_sublayer(n, l)
        else:
            for i, l in enumerate(layers):
                self.add_sublayer(str(i), l)

    def __getitem__(self, idx):
        vals = list(self._sub_layers.values())
        if isinstance(idx, slice):
            return Sequential(*vals[idx])
        if isinstance(idx, str):
            return self._sub_layers[idx]
        return vals[idx]

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers.values())

    def forward(self, x):
        for l in self._sub_layers.values():
            x = l(x)
        return x


class LayerList(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        if sublayers is not None:
            for i, l in enumerate(sublayers):
                self.add_sublayer(str(i), l)

    def __getitem__(self, idx):
        vals = list(self._sub_layers.values())
        if isinstance(idx, slice):
            return LayerList(vals[idx])
        return vals[idx]

    def __setitem__(self, idx, layer):
        self._sub_layers[list(self._sub_layers)[idx]] = layer

    def __delitem__(self, idx):
        keys = list(self._sub_layers)
        del self._sub_layers[keys[idx]]
        vals = list(self._sub_layers.values())
        self._sub_layers.clear()
        for i, l in enumerate(vals):
            self._sub_layers[str(i)] = l

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers.values())

    def append(self, layer):
        self.add_sublayer(str(len(self)), layer)
        return self

    def extend(self, layers):
        for l in layers:
            self.append(l)
        return self

    def insert(self, index, layer):
        vals = list(self._sub_layers.values())
        vals.insert(index, layer)
        self._sub_layers.clear()
        for i, l in enumerate(vals):
            self._sub_layers[str(i)] = l


class LayerDict(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        if sublayers is not None:
            self.update(sublayers)

    def __getitem__(self, k):
        return self._sub_layers[k]

    def __setitem__(self, k, v):
        self.add_sublayer(k, v)

    def __delitem__(self, k):
        del self._sub_layers[k]

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers)

    def __contains__(self, k):
        return k in self._sub_layers

    def keys(self):
        return self._sub_layers.keys()

    def values(self):
        return self._sub_layers.values()

    def items(self):
        return self._sub_layers.items()

    def update(self, sublayers):
        items = sublayers.items() if hasattr(sublayers, 'items') else sublayers
        for k, v in items:
            self.add_sublayer(k, v)

    def pop(self, k):
        return self._sub_layers.pop(k)

    def clear(self):
        self._sub_layers.clear()


class ParameterList(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        if parameters is not None:
            for i, p in enumerate(parameters):
                self.add_parameter(str(i), p)

    def __getitem__(self, i):
        return list(self._parameters.values())[i]

    def __setitem__(self, i, p):
        self._parameters[str(i)] = p

    def __len__(self):
        return len(self._parameters)

    def __iter__(self):
        return iter(self._parameters.values())

    def append(self, p):
        self.add_parameter(str(len(self)), p)
        return self
