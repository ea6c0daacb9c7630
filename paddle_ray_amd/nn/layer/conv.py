"""Convolution + pooling layers (parity: python/paddle/nn/layer/{conv,pooling}.py).

Conv weights keep paddle's [out, in/groups, *k] layout (transpose: [in, out/groups, *k]).
Default init = Normal(0, sqrt(2 / fan_in)) like the reference's
``_get_default_param_initializer``.
"""
import math

import numpy as np

from .. import functional as F
from .. import initializer as I
from .layers import Layer


def _ntuple(v, n):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


class _ConvNd(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, transposed, dims, stride=1,
                 padding=0, padding_mode='zeros', output_padding=0, dilation=1, groups=1,
                 weight_attr=None, bias_attr=None, data_format='NCHW'):
        super().__init__()
        self._in_channels, self._out_channels = in_channels, out_channels
        self._kernel_size = _ntuple(kernel_size, dims)
        self._stride, self._padding = stride, padding
        self._padding_mode = padding_mode
        self._output_padding, self._dilation, self._groups = output_padding, dilation, groups
        self._data_format = data_format
        self._transposed = transposed
        self._dims = dims
        if transposed:
            shape = [in_channels, out_channels // groups] + list(self._kernel_size)
        else:
            shape = [out_channels, in_channels // groups] + list(self._kernel_size)
        fan_in = (in_channels // groups) * int(np.prod(self._kernel_size))
        std = math.sqrt(2.0 / fan_in)
        self.weight = self.create_parameter(shape, weight_attr, default_initializer=I.Normal(0.0, std))
        self.bias = self.create_parameter([out_channels], bias_attr, is_bias=True)

    def _pad_input(self, x):
        if self._padding_mode != 'zeros':
            p = _ntuple(self._padding, self._dims)
            pads = []
            for v in reversed(p):
                pads += [v, v]
            mode = {'reflect': 'reflect', 'replicate': 'replicate', 'circular': 'circular'}[
                self._padding_mode]
            return F.pad(x, pads, mode, data_format=self._data_format), 0
        return x, self._padding

    def extra_repr(self):
        return (f'{self._in_channels}, {self._out_channels}, kernel_size={list(self._kernel_size)}, '
                f'stride={self._stride}, padding={self._padding}, data_format={self._data_format}')


class Conv1D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, padding_mode='zeros', weight_attr=None, bias_attr=None,
                 data_format='NCL'):
        super().__init__(in_channels, out_channels, kernel_size, False, 1, stride, padding,
                         padding_mode, 0, dilation, groups, weight_attr, bias_attr, data_format)

    def forward(self, x):
        x, p = self._pad_input(x)
        return F.conv1d(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups,
                        self._data_format)


class Conv2D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, padding_mode='zeros', weight_attr=None, bias_attr=None,
                 data_format='NCHW'):
        super().__init__(in_channels, out_channels, kernel_size, False, 2, stride, padding,
                         padding_mode, 0, dilation, groups, weight_attr, bias_attr, data_format)

    def forward(self, x):
        x, p = self._pad_input(x)
        return F.conv2d(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups,
                        self._data_format)


class Conv3D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, padding_mode='zeros', weight_attr=None, bias_attr=None,
                 data_format='NCDHW'):
        super().__init__(in_channels, out_channels, kernel_size, False, 3, stride, padding,
                         padding_mode, 0, dilation, groups, weight_attr, bias_attr, data_format)

    def forward(self, x):
        x, p = self._pad_input(x)
        return F.conv3d(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups,
                        self._data_format)


class Conv1DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 output_padding=0, groups=1, dilation=1, weight_attr=None, bias_attr=None,
                 data_format='NCL'):
        super().__init__(in_channels, out_channels, kernel_size, True, 1, stride, padding, 'zeros',
                         output_padding, dilation, groups, weight_attr, bias_attr, data_format)

    def forward(self, x, output_size=None):
        return F.conv1d_transpose(x, self.weight, self.bias, self._stride, self._padding,
                                  self._output_padding, self._groups, self._dilation, output_size,
                                  self._data_format)


class Conv2DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 output_padding=0, dilation=1, groups=1, weight_attr=None, bias_attr=None,
                 data_format='NCHW'):
        super().__init__(in_channels, out_channels, kernel_size, True, 2, stride, padding, 'zeros',
                         output_padding, dilation, groups, weight_attr, bias_attr, data_format)

    def forward(self, x, output_size=None):
        return F.conv2d_transpose(x, self.weight, self.bias, self._stride, self._padding,
                                  self._output_padding, self._dilation, self._groups, output_size,
                                  self._data_format)


class Conv3DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 output_padding=0, dilation=1, groups=1, weight_attr=None, bias_attr=None,
                 data_format='NCDHW'):
        super().__init__(in_channels, out_channels, kernel_size, True, 3, stride, padding, 'zeros',
                         output_padding, dilation, groups, weight_attr, bias_attr, data_format)

    def forward(self, x, output_size=None):
        return F.conv3d_transpose(x, self.weight, self.bias, self._stride, self._padding,
                                  self._output_padding, self._groups, self._dilation, output_size,
                                  self._data_format)


# -- pooling -------------------------------------------------------------------------
class _Pool(Layer):
    def __init__(self, fn, **kw):
        super().__init__()
        self._fn, self._kw = fn, kw

    def forward(self, x):
        return self._fn(x, **self._kw)

    def extra_repr(self):
        return ', '.join(f'{k}={v}' for k, v in self._kw.items())


class MaxPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 name=None):
        super().__init__(F.max_pool1d, kernel_size=kernel_size, stride=stride, padding=padding,
                         return_mask=return_mask, ceil_mode=ceil_mode)


class MaxPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format='NCHW', name=None):
        super().__init__(F.max_pool2d, kernel_size=kernel_size, stride=stride, padding=padding,
                         return_mask=return_mask, ceil_mode=ceil_mode, data_format=data_format)


class MaxPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format='NCDHW', name=None):
        super().__init__(F.max_pool3d, kernel_size=kernel_size, stride=stride, padding=padding,
                         return_mask=return_mask, ceil_mode=ceil_mode, data_format=data_format)


class AvgPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False,
                 name=None):
        super().__init__(F.avg_pool1d, kernel_size=kernel_size, stride=stride, padding=padding,
                         exclusive=exclusive, ceil_mode=ceil_mode)


class AvgPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
                 divisor_override=None, data_format='NCHW', name=None):
        super().__init__(F.avg_pool2d, kernel_size=kernel_size, stride=stride, padding=padding,
                         ceil_mode=ceil_mode, exclusive=exclusive,
                         divisor_override=divisor_override, data_format=data_format)


class AvgPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
                 divisor_override=None, data_format='NCDHW', name=None):
        super().__init__(F.avg_pool3d, kernel_size=kernel_size, stride=stride, padding=padding,
                         ceil_mode=ceil_mode, exclusive=exclusive,
                         divisor_override=divisor_override, data_format=data_format)


class AdaptiveAvgPool1D(_Pool):
    def __init__(self, output_size, name=None):
        super().__init__(F.adaptive_avg_pool1d, output_size=output_size)


class AdaptiveAvgPool2D(_Pool):
    def __init__(self, output_size, data_format='NCHW', name=None):
        super().__init__(F.adaptive_avg_pool2d, output_size=output_size, data_format=data_format)


class AdaptiveAvgPool3D(_Pool):
    def __init__(self, output_size, data_format='NCDHW', name=None):
        super().__init__(F.adaptive_avg_pool3d, output_size=output_size, data_format=data_format)


class AdaptiveMaxPool1D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(F.adaptive_max_pool1d, output_size=output_size, return_mask=return_mask)


class AdaptiveMaxPool2D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(F.adaptive_max_pool2d, output_size=output_size, return_mask=return_mask)


class AdaptiveMaxPool3D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(F.adaptive_max_pool3d, output_size=output_size, return_mask=return_mask)


class MaxUnPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, data_format='NCL', output_size=None,
                 name=None):
        super().__init__(None)
        self.a = (kernel_size, stride, padding, data_format, output_size)

    def forward(self, x, indices):
        return F.max_unpool1d(x, indices, *self.a)


class MaxUnPool2D(MaxUnPool1D):
    def forward(self, x, indices):
        return F.max_unpool2d(x, indices, *self.a)


class MaxUnPool3D(MaxUnPool1D):
    def forward(self, x, indices):
        return F.max_unpool3d(x, indices, *self.a)
