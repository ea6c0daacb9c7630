"""paddle.incubate.operators (parity: python/paddle/incubate/operators/__init__.py).

``resnet_unit`` / ``ResNetUnit`` (reference: incubate/operators/resnet_unit.py:25,150 over
fluid/operators/fused/resnet_unit_op.cu, a cuDNN-v8 fused conv + BN-statistics graph) is
built here from the two gfx950 pieces the ResNet path already uses:

* the convolution runs channels-last on the in-tree implicit-GEMM MFMA kernel
  (``ops/fused.py`` ConvKxKFn / Conv1x1Fn; the im2col rows are gathered by LDS-DMA, never
  materialised) — the NHWC filter ``[Cout, KH, KW, Cin]`` is exactly the kernel's OHWI
  operand, so no weight copy is made;
* the BatchNorm (+ residual add + ReLU) is ONE statistics pass plus ONE apply pass of
  ``ops/csrc/bn.hip`` (``fused_bn_add_act``), which also writes the ReLU keep-bits the
  backward reads instead of the output.

``has_shortcut`` runs the shortcut conv + BN with identity activation and feeds it to the
main BN's fused residual add; ``fuse_add`` adds ``z`` directly. ``use_global_stats`` /
``is_test`` normalise with the running statistics.
"""
import torch

from ...framework.core import Tensor, _u
from ...nn import functional as F
from ...nn import initializer as I
from ...nn.layer.layers import Layer, ParamAttr
from .. import softmax_mask_fuse, softmax_mask_fuse_upper_triangle, graph_khop_sampler  # noqa: F401
from ...geometric import (send_u_recv as graph_send_recv, reindex_graph as graph_reindex,  # noqa: F401
                          sample_neighbors as graph_sample_neighbors)

__all__ = ['ResNetUnit', 'resnet_unit', 'unzip', 'softmax_mask_fuse',
           'softmax_mask_fuse_upper_triangle', 'graph_send_recv', 'graph_khop_sampler',
           'graph_sample_neighbors', 'graph_reindex']


def _bn_vec(p):
    """[1,1,1,C] / [1,C,1,1] BN parameter -> [C] view (gradients and in-place running-stat
    updates reach the parameter's storage)."""
    return None if p is None else _u(p).reshape(-1)


def _conv_bn(x, filt, scale, bias, mean, var, z, stride, padding, dilation, groups, momentum,
             eps, training, act):
    """act(BN(conv(x)) + z) on channels-last tensors, filt in OHWI. Training KxK convolutions on
    the device take the BN statistics from the convolution's epilogue (ops.fused.conv_bn_act_nhwc)."""
    from ...ops import fused as K
    w = _u(filt).permute(0, 3, 1, 2)  # OIHW-shaped view of the OHWI storage
    xt, rm = _u(x), _bn_vec(mean)
    if (dilation == 1 and groups == 1 and isinstance(stride, int) and isinstance(padding, int)
            and xt.dtype == w.dtype and K.conv_bn_stats_ok(xt, w, stride, padding, rm, training)):
        return K.conv_bn_act_nhwc(xt, w, stride, padding, _bn_vec(scale), _bn_vec(bias), rm,
                                  _bn_vec(var), training, momentum, eps,
                                  _u(z) if z is not None else None, act == 'relu')
    c = F.conv2d(x, w, None, stride, padding, dilation, groups, data_format='NHWC')
    return F.fused_bn_add_act(c, z, _bn_vec(mean), _bn_vec(var), _bn_vec(scale), _bn_vec(bias),
                              training, momentum, eps, act, data_format='NHWC')


def resnet_unit(x, filter_x, scale_x, bias_x, mean_x, var_x, z, filter_z, scale_z, bias_z, mean_z,
                var_z, stride, stride_z, padding, dilation, groups, momentum, eps, data_format,
                fuse_add, has_shortcut, use_global_stats, is_test, act):
    """y = act(BN_x(conv(x, filter_x)) + shortcut) where shortcut is BN_z(conv(z, filter_z))
    when ``has_shortcut``, ``z`` when ``fuse_add`` and 0 otherwise (reference
    resnet_unit.py:25 / resnet_unit_op.cc). Filters are OHWI for NHWC (OIHW for NCHW);
    running statistics are updated in place with paddle's momentum convention."""
    if act not in (None, 'relu', 'identity', ''):
        raise ValueError(f"resnet_unit: unsupported act_type {act!r}")
    act = 'relu' if act == 'relu' else None
    if groups != 1:
        raise ValueError("resnet_unit: groups must be 1")
    training = not (use_global_stats or is_test)
    nchw = data_format == 'NCHW'
    xt = _u(x)
    zt = _u(z) if z is not None else None
    fx, fz = filter_x, filter_z
    if nchw:  # run channels-last: activations NHWC, filters OIHW -> OHWI views
        xt = xt.permute(0, 2, 3, 1)
        zt = zt.permute(0, 2, 3, 1) if zt is not None else None
        fx = _u(fx).permute(0, 2, 3, 1)
        fz = _u(fz).permute(0, 2, 3, 1) if fz is not None else None
    short = None
    if has_shortcut:
        if zt is None or fz is None:
            raise ValueError("resnet_unit: has_shortcut needs z and filter_z")
        short = _u(_conv_bn(zt, fz, scale_z, bias_z, mean_z, var_z, None, stride_z, padding, dilation,
                            groups, momentum, eps, training, None))
    elif fuse_add:
        if zt is None:
            raise ValueError("resnet_unit: fuse_add needs z")
        short = zt
    y = _u(_conv_bn(xt, fx, scale_x, bias_x, mean_x, var_x, short, stride, padding, dilation,
                    groups, momentum, eps, training, act))
    if nchw:
        y = y.permute(0, 3, 1, 2)
    return Tensor(y)


class ResNetUnit(Layer):
    """Fused conv + BN (+ shortcut conv + BN | + residual) + activation block (reference
    incubate/operators/resnet_unit.py:150; same constructor, parameter shapes and
    initialisers: filters ~ N(0, sqrt(2 / (k*k*Cin))), BN scale 1 / bias 0, running mean 0 /
    var 1 as non-trainable fp32 parameters)."""

    def __init__(self, num_channels_x, num_filters, filter_size, stride=1, momentum=0.9, eps=1e-5,
                 data_format='NHWC', act='relu', fuse_add=False, has_shortcut=False,
                 use_global_stats=False, is_test=False, filter_x_attr=None, scale_x_attr=None,
                 bias_x_attr=None, moving_mean_x_name=None, moving_var_x_name=None,
                 num_channels_z=1, stride_z=1, filter_z_attr=None, scale_z_attr=None,
                 bias_z_attr=None, moving_mean_z_name=None, moving_var_z_name=None):
        super().__init__()
        if data_format not in ('NHWC', 'NCHW'):
            raise ValueError(f"conv_format must be one of {{'NHWC', 'NCHW'}}, but got "
                             f"conv_format='{data_format}'")
        self._stride, self._stride_z, self._dilation = stride, stride_z, 1
        self._padding = (filter_size - 1) // 2
        self._groups, self._momentum, self._eps = 1, momentum, eps
        self._data_format, self._act = data_format, act
        self._fuse_add, self._has_shortcut = fuse_add, has_shortcut
        self._use_global_stats, self._is_test = use_global_stats, is_test
        k = filter_size
        nchw = data_format == 'NCHW'
        bn_shape = [1, num_filters, 1, 1] if nchw else [1, 1, 1, num_filters]

        def fshape(cin):
            return [num_filters, cin, k, k] if nchw else [num_filters, k, k, cin]

        def finit(cin):
            return I.Normal(0.0, (2.0 / (k * k * cin)) ** 0.5)

        def stat(name, v):
            p = self.create_parameter(bn_shape, ParamAttr(name=name, initializer=I.Constant(v),
                                                          trainable=False), dtype='float32')
            p.stop_gradient = True
            return p

        self.filter_x = self.create_parameter(fshape(num_channels_x), filter_x_attr,
                                              default_initializer=finit(num_channels_x))
        self.scale_x = self.create_parameter(bn_shape, scale_x_attr, dtype='float32',
                                             default_initializer=I.Constant(1.0))
        self.bias_x = self.create_parameter(bn_shape, bias_x_attr, dtype='float32', is_bias=True)
        self.mean_x = stat(moving_mean_x_name, 0.0)
        self.var_x = stat(moving_var_x_name, 1.0)
        if has_shortcut:
            self.filter_z = self.create_parameter(fshape(num_channels_z), filter_z_attr,
                                                  default_initializer=finit(num_channels_z))
            self.scale_z = self.create_parameter(bn_shape, scale_z_attr, dtype='float32',
                                                 default_initializer=I.Constant(1.0))
            self.bias_z = self.create_parameter(bn_shape, bias_z_attr, dtype='float32',
                                                is_bias=True)
            self.mean_z = stat(moving_mean_z_name, 0.0)
            self.var_z = stat(moving_var_z_name, 1.0)
        else:
            self.filter_z = self.scale_z = self.bias_z = self.mean_z = self.var_z = None

    def forward(self, x, z=None):
        if self._fuse_add and z is None:
            raise ValueError("z can not be None")
        return resnet_unit(x, self.filter_x, self.scale_x, self.bias_x, self.mean_x, self.var_x,
                           z, self.filter_z, self.scale_z, self.bias_z, self.mean_z, self.var_z,
                           self._stride, self._stride_z, self._padding, self._dilation,
                           self._groups, self._momentum, self._eps, self._data_format,
                           self._fuse_add, self._has_shortcut, self._use_global_stats,
                           self._is_test or not self.training, self._act)


def unzip(input, lod):
    """Scatter the rows of a zipped [N, M] tensor back to the K-1 sequences described by
    ``lod`` (reference incubate/operators/unzip.py:19, unzip_op.cu): sequence i receives the
    next zipped row when lod[i+1] > lod[i] (its length must equal M) and zeros otherwise."""
    x, lo = _u(input), _u(lod).to(torch.int64)
    lens = lo[1:] - lo[:-1]
    nonempty = lens > 0
    if x.numel() and bool((lens[nonempty] != x.shape[1]).any()):
        raise ValueError("unzip: every non-empty lod segment must span exactly M columns")
    out = torch.zeros((lens.numel(), x.shape[1]), dtype=x.dtype, device=x.device)
    src = torch.cumsum(nonempty.to(torch.int64), 0) - 1
    out[nonempty] = x[src[nonempty]]
    return Tensor(out)
