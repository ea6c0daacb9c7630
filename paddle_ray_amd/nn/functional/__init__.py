"""paddle.nn.functional (parity: python/paddle/nn/functional/*.py).

Hot ops route to the HIP kernel registry (``ops.fused``): layer_norm,
rms_norm, softmax (last axis), softmax_with_cross_entropy / cross_entropy
(hard labels), gelu(+bias), flash/scaled-dot-product attention. GEMM/conv go to
hipBLASLt / MIOpen through PyTorch-ROCm.
"""
import math
import os

import numpy as np
import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _u, convert_dtype
from ...ops import fused as K
from ...amp import amp_op as _amp_op


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _w(t):
    return Tensor(t)


def _opt(x):
    return None if x is None else _t(x)


# =============================================================================
# activations
# =============================================================================
@_amp_op('relu')
def relu(x, name=None):
    return _w(torch.relu(_t(x)))


def relu_(x, name=None):
    torch.relu_(x._t)
    return x


def relu6(x, name=None):
    return _w(TF.relu6(_t(x)))


def leaky_relu(x, negative_slope=0.01, name=None):
    return _w(TF.leaky_relu(_t(x), negative_slope))


def elu(x, alpha=1.0, name=None):
    return _w(TF.elu(_t(x), alpha))


def elu_(x, alpha=1.0, name=None):
    TF.elu_(x._t, alpha)
    return x


def celu(x, alpha=1.0, name=None):
    return _w(TF.celu(_t(x), alpha))


def selu(x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717,
         name=None):
    t = _t(x)
    return _w(scale * torch.where(t > 0, t, alpha * (torch.exp(t) - 1)))


@_amp_op('gelu')
def gelu(x, approximate=False, name=None):
    t = _t(x)
    if t.is_cuda:
        return _w(K.bias_gelu(t, None, bool(approximate)))
    return _w(TF.gelu(t, approximate='tanh' if approximate else 'none'))


def fused_bias_gelu(x, bias, approximate=False):
    return _w(K.bias_gelu(_t(x), _t(bias), bool(approximate)))


def silu(x, name=None):
    return _w(TF.silu(_t(x)))


def swish(x, name=None):
    return _w(TF.silu(_t(x)))


def mish(x, name=None):
    return _w(TF.mish(_t(x)))


@_amp_op('sigmoid')
def sigmoid(x, name=None):
    return _w(torch.sigmoid(_t(x)))


def tanh(x, name=None):
    return _w(torch.tanh(_t(x)))


def tanh_(x, name=None):
    x._t.tanh_()
    return x


def hardtanh(x, min=-1.0, max=1.0, name=None):
    return _w(TF.hardtanh(_t(x), min, max))


def hardsigmoid(x, slope=0.1666667, offset=0.5, name=None):
    return _w(torch.clamp(_t(x) * slope + offset, 0, 1))


def hardswish(x, name=None):
    return _w(TF.hardswish(_t(x)))


def hardshrink(x, threshold=0.5, name=None):
    return _w(TF.hardshrink(_t(x), threshold))


def softshrink(x, threshold=0.5, name=None):
    return _w(TF.softshrink(_t(x), threshold))


def softsign(x, name=None):
    return _w(TF.softsign(_t(x)))


def softplus(x, beta=1, threshold=20, name=None):
    return _w(TF.softplus(_t(x), beta, threshold))


def tanhshrink(x, name=None):
    return _w(TF.tanhshrink(_t(x)))


def thresholded_relu(x, threshold=1.0, name=None):
    t = _t(x)
    return _w(torch.where(t > threshold, t, torch.zeros_like(t)))


def log_sigmoid(x, name=None):
    return _w(TF.logsigmoid(_t(x)))


def prelu(x, weight, data_format='NCHW', name=None):
    t, w = _t(x), _t(weight)
    if w.numel() > 1 and data_format in ('NHWC', 'NLC', 'NDHWC'):
        return _w(torch.where(t >= 0, t, t * w))
    return _w(TF.prelu(t, w))


def rrelu(x, lower=1. / 8., upper=1. / 3., training=True, name=None):
    return _w(TF.rrelu(_t(x), lower, upper, training))


def maxout(x, groups, axis=1, name=None):
    t = _t(x)
    shp = list(t.shape)
    c = shp[axis]
    shp[axis:axis + 1] = [c // groups, groups]
    return _w(t.reshape(shp).amax(axis + 1))


def glu(x, axis=-1, name=None):
    return _w(TF.glu(_t(x), axis))


@_amp_op('softmax')
def softmax(x, axis=-1, dtype=None, name=None):
    t = _t(x)
    if dtype is not None:
        t = t.to(convert_dtype(dtype))
    if t.is_cuda and (axis == -1 or axis == t.dim() - 1):
        return _w(K.softmax_lastdim(t))
    return _w(torch.softmax(t, axis))


def softmax_(x, axis=-1, dtype=None, name=None):
    r = softmax(x, axis, dtype)
    object.__setattr__(x, '_t', r._t)
    return x


@_amp_op('log_softmax')
def log_softmax(x, axis=-1, dtype=None, name=None):
    t = _t(x)
    if dtype is not None:
        t = t.to(convert_dtype(dtype))
    return _w(torch.log_softmax(t, axis))


def gumbel_softmax(x, temperature=1.0, hard=False, axis=-1, name=None):
    return _w(TF.gumbel_softmax(_t(x), tau=temperature, hard=hard, dim=axis))


# =============================================================================
# common
# =============================================================================
@_amp_op('linear')
def linear(x, weight, bias=None, name=None):
    """y = x @ W + b with paddle's [in, out] weight layout (hipBLASLt GEMM)."""
    t, w = _t(x), _t(weight)
    if w.dim() == 2 and t.dim() >= 2 and t.dtype == w.dtype:
        from ...ops import fused as _K
        return _w(_K.linear(t, w, None if bias is None else _t(bias)))
    if bias is not None:
        b = _t(bias)
        if t.dim() == 2:
            return _w(torch.addmm(b, t, w))
        return _w(torch.addmm(b, t.reshape(-1, t.shape[-1]), w).reshape(*t.shape[:-1], w.shape[-1]))
    return _w(torch.matmul(t, w))


def bilinear(x1, x2, weight, bias=None, name=None):
    return _w(TF.bilinear(_t(x1), _t(x2), _t(weight), None if bias is None else _t(bias).flatten()))


def dropout(x, p=0.5, axis=None, training=True, mode='upscale_in_train', name=None):
    t = _t(x)
    if not training or p == 0:
        if mode == 'downscale_in_infer' and not training:
            return _w(t * (1 - p))
        return x if isinstance(x, Tensor) else _w(t)
    if axis is not None:
        axes = [axis] if isinstance(axis, int) else list(axis)
        mshape = [t.shape[i] if i in [a % t.dim() for a in axes] else 1 for i in range(t.dim())]
        mask = (torch.rand(mshape, device=t.device) >= p).to(t.dtype)
        out = t * mask
        return _w(out / (1 - p) if mode == 'upscale_in_train' else out)
    if mode == 'upscale_in_train':
        return _w(TF.dropout(t, p, True))
    return _w(t * (torch.rand_like(t, dtype=torch.float32) >= p).to(t.dtype))


def dropout2d(x, p=0.5, training=True, data_format='NCHW', name=None):
    t = _t(x)
    if data_format == 'NHWC':
        return _w(TF.dropout2d(t.permute(0, 3, 1, 2), p, training).permute(0, 2, 3, 1))
    return _w(TF.dropout2d(t, p, training))


def dropout3d(x, p=0.5, training=True, data_format='NCDHW', name=None):
    return _w(TF.dropout3d(_t(x), p, training))


def alpha_dropout(x, p=0.5, training=True, name=None):
    return _w(TF.alpha_dropout(_t(x), p, training))


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    t = _t(label)
    n = t.shape[-1]
    pd = (1.0 / n) if prior_dist is None else _t(prior_dist)
    return _w((1 - epsilon) * t + epsilon * pd)


def one_hot(x, num_classes, name=None):
    return _w(TF.one_hot(_t(x).long(), num_classes).float())


def embedding(x, weight, padding_idx=None, sparse=False, name=None):
    """Row lookup (gfx950 kernel on the device; rows of ``padding_idx`` read as zeros and
    receive no gradient, as in paddle's lookup_table_v2)."""
    w = _t(weight)
    if padding_idx is not None and padding_idx < 0:
        padding_idx += w.shape[0]
    return _w(K.embedding(_t(x).long(), w, padding_idx))


def pad(x, pad, mode='constant', value=0.0, data_format='NCHW', name=None):
    t = _t(x)
    if isinstance(pad, Tensor):
        pad = pad.tolist()
    pad = list(pad)
    nd = t.dim()
    if len(pad) == 2 * nd:
        # paddle full-rank pad: [d0_before, d0_after, d1_before, ...] -> torch reversed pairs
        tp = []
        for i in reversed(range(nd)):
            tp += [pad[2 * i], pad[2 * i + 1]]
        return _w(TF.pad(t, tp, mode=mode if mode != 'edge' else 'replicate', value=value))
    channel_last = data_format in ('NHWC', 'NLC', 'NDHWC')
    if channel_last:
        t = t.movedim(-1, 1)
    # paddle pads spatial dims as [left, right, top, bottom, front, back] (last dim first)
    m = {'constant': 'constant', 'reflect': 'reflect', 'replicate': 'replicate', 'edge': 'replicate',
         'circular': 'circular'}[mode]
    out = TF.pad(t, pad, mode=m, value=value) if m == 'constant' else TF.pad(t, pad, mode=m)
    if channel_last:
        out = out.movedim(1, -1)
    return _w(out)


def zeropad2d(x, padding, data_format='NCHW', name=None):
    if isinstance(padding, int):
        padding = [padding] * 4
    return pad(x, padding, 'constant', 0.0, data_format)


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return _w(TF.cosine_similarity(_t(x1), _t(x2), axis, eps))


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    return _w(TF.pairwise_distance(_t(x), _t(y), p, epsilon, keepdim))


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return _w(TF.normalize(_t(x), p, axis, epsilon))


def interpolate(x, size=None, scale_factor=None, mode='nearest', align_corners=False,
                align_mode=0, data_format='NCHW', name=None):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC')
    if cl:
        t = t.movedim(-1, 1)
    if isinstance(size, Tensor):
        size = size.tolist()
    if isinstance(size, (list, tuple)):
        size = [int(s.item()) if isinstance(s, Tensor) else int(s) for s in size]
    m = {'nearest': 'nearest', 'bilinear': 'bilinear', 'trilinear': 'trilinear', 'bicubic': 'bicubic',
         'linear': 'linear', 'area': 'area'}[mode.lower()]
    kw = {} if m in ('nearest', 'area') else {'align_corners': align_corners}
    out = TF.interpolate(t, size=size, scale_factor=scale_factor, mode=m, **kw)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


upsample = interpolate


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    if isinstance(paddings, (list, tuple)) and len(paddings) == 4:
        t = TF.pad(_t(x), [paddings[1], paddings[3], paddings[0], paddings[2]])
        return _w(TF.unfold(t, kernel_sizes, dilations, 0, strides))
    return _w(TF.unfold(_t(x), kernel_sizes, dilations, paddings, strides))


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return _w(TF.fold(_t(x), output_sizes, kernel_sizes, dilations, paddings, strides))


def pixel_shuffle(x, upscale_factor, data_format='NCHW', name=None):
    t = _t(x)
    if data_format == 'NHWC':
        return _w(TF.pixel_shuffle(t.permute(0, 3, 1, 2), upscale_factor).permute(0, 2, 3, 1))
    return _w(TF.pixel_shuffle(t, upscale_factor))


def pixel_unshuffle(x, downscale_factor, data_format='NCHW', name=None):
    t = _t(x)
    if data_format == 'NHWC':
        return _w(TF.pixel_unshuffle(t.permute(0, 3, 1, 2), downscale_factor).permute(0, 2, 3, 1))
    return _w(TF.pixel_unshuffle(t, downscale_factor))


def channel_shuffle(x, groups, data_format='NCHW', name=None):
    t = _t(x)
    if data_format == 'NHWC':
        return _w(TF.channel_shuffle(t.permute(0, 3, 1, 2), groups).permute(0, 2, 3, 1))
    return _w(TF.channel_shuffle(t, groups))


def affine_grid(theta, out_shape, align_corners=True, name=None):
    if isinstance(out_shape, Tensor):
        out_shape = out_shape.tolist()
    return _w(TF.affine_grid(_t(theta), list(out_shape), align_corners))


def grid_sample(x, grid, mode='bilinear', padding_mode='zeros', align_corners=True, name=None):
    return _w(TF.grid_sample(_t(x), _t(grid), mode, padding_mode, align_corners))


def sequence_mask(x, maxlen=None, dtype='int64', name=None):
    t = _t(x)
    maxlen = int(t.max().item()) if maxlen is None else int(maxlen)
    r = torch.arange(maxlen, device=t.device)
    return _w((r < t.unsqueeze(-1)).to(convert_dtype(dtype)))


def diag_embed(input, offset=0, dim1=-2, dim2=-1):
    return _w(torch.diag_embed(_t(input), offset, dim1, dim2))


def temporal_shift(x, seg_num, shift_ratio=0.25, name=None, data_format='NCHW'):
    t = _t(x)
    nt, c, h, w = t.shape
    n = nt // seg_num
    t = t.reshape(n, seg_num, c, h, w)
    fold = int(c * shift_ratio)
    out = torch.zeros_like(t)
    out[:, :-1, :fold] = t[:, 1:, :fold]
    out[:, 1:, fold:2 * fold] = t[:, :-1, fold:2 * fold]
    out[:, :, 2 * fold:] = t[:, :, 2 * fold:]
    return _w(out.reshape(nt, c, h, w))


# =============================================================================
# conv / pool
# =============================================================================
def _ntuple(v, n):
    if isinstance(v, (list, tuple)):
        return tuple(v) if len(v) == n else tuple(v) * (n // len(v))
    return (v,) * n


def _conv_padding(padding, n, t=None, ksize=None, stride=None, dilation=None):
    if isinstance(padding, str):
        p = padding.upper()
        if p == 'VALID':
            return 0, None
        if p == 'SAME':
            return 'same', None
    if isinstance(padding, (list, tuple)):
        padding = list(padding)
        if len(padding) == 2 * n and not isinstance(padding[0], (list, tuple)):
            if all(padding[2 * i] == padding[2 * i + 1] for i in range(n)):
                return tuple(padding[0::2]), None
            tp = []
            for i in reversed(range(n)):
                tp += [padding[2 * i], padding[2 * i + 1]]
            return 0, tp
        if len(padding) == n + 2 and isinstance(padding[0], (list, tuple)):
            sp = [p for p in padding if list(p) != [0, 0]]
            padding = [x for p in padding[2:] for x in p] if len(sp) <= n else sp
            return _conv_padding(padding, n)
    return _ntuple(padding, n), None


# 1x1 channels-last convs: 'mfma' = GEMMs with the in-tree split-K MFMA kernel for dgrad /
# wgrad (ops/fused.py Conv1x1Fn; default: ResNet50 7596 vs 7485 img/s with MIOpen, A/B on one
# box), 'blas' = one hipBLASLt GEMM per direction (round-1 A/B:
# no split-K for the huge-K wgrad), 'miopen' = MIOpen's implicit-GEMM kernels
_CONV1X1 = os.environ.get('PRA_CONV1X1', 'mfma')
_CONV1X1_GEMM = _CONV1X1 == 'blas' or os.environ.get('PRA_CONV1X1_GEMM', '0') == '1'
# KxK channels-last convs (groups 1, Cin % 64 == 0): 'mfma' = implicit GEMM on the in-tree
# LDS-DMA kernel for forward and stride-1 dgrad (ops/fused.py ConvKxKFn; default: ResNet50
# 7983 vs 7793 img/s, profiles/r2_conv), 'miopen' = MIOpen for every direction
_CONVKXK = os.environ.get('PRA_CONVKXK', 'mfma')


def _conv1x1_gemm(t, w, bias, st):
    """Channels-last 1x1 conv (pad 0, dilation 1, groups 1) as one hipBLASLt GEMM
    [N*Ho*Wo, Cin] @ [Cin, Cout]: dgrad and wgrad are plain GEMMs too (no split-K atomics,
    no workspace zero-fill), and the NHWC activation is read in place."""
    if st != (1, 1):
        t = t[:, ::st[0], ::st[1], :]
    n, h, wd, cin = t.shape
    cout = w.shape[0]
    y = torch.mm(t.reshape(-1, cin), w.view(cout, cin).t())
    if bias is not None:
        y = y + bias
    return y.view(n, h, wd, cout)


def _conv(fn, n, x, weight, bias, stride, padding, dilation, groups, data_format):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC')
    pad_, extra = _conv_padding(padding, n)
    if ((_CONV1X1_GEMM or _CONV1X1 == 'mfma') and n == 2 and cl and t.is_cuda and groups == 1
            and extra is None and _t(weight).shape[2:] == (1, 1) and _ntuple(dilation, 2) == (1, 1)
            and pad_ in (0, (0, 0), [0, 0]) and t.dtype == _t(weight).dtype):
        if _CONV1X1 == 'mfma' and t.dtype in (torch.bfloat16, torch.float16):
            return _w(K.conv1x1_nhwc(t, _t(weight), None if bias is None else _t(bias),
                                     _ntuple(stride, 2)))
        return _w(_conv1x1_gemm(t, _t(weight), None if bias is None else _t(bias),
                                _ntuple(stride, 2)))
    if (_CONVKXK == 'mfma' and n == 2 and cl and t.is_cuda and groups == 1 and extra is None
            and _ntuple(dilation, 2) == (1, 1)):
        st, pd = _ntuple(stride, 2), _ntuple(pad_, 2) if not isinstance(pad_, str) else None
        w = _t(weight)
        if (pd is not None and st[0] == st[1] and pd[0] == pd[1] and w.shape[2] == w.shape[3] > 1
                and K.conv_kxk_supported(t, w, st[0], pd[0])):
            return _w(K.conv_kxk_nhwc(t, w, None if bias is None else _t(bias), st[0], pd[0]))
    if cl:
        t = t.movedim(-1, 1)
    if extra is not None:
        t = TF.pad(t, extra)
    w = _t(weight)
    if t.dtype != w.dtype:
        t = t.to(w.dtype)
    out = fn(t, w, None if bias is None else _t(bias), _ntuple(stride, n), pad_,
             _ntuple(dilation, n), groups)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


@_amp_op('conv1d')
def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format='NCL',
           name=None):
    return _conv(TF.conv1d, 1, x, weight, bias, stride, padding, dilation, groups, data_format)


@_amp_op('conv2d')
def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format='NCHW',
           name=None):
    return _conv(TF.conv2d, 2, x, weight, bias, stride, padding, dilation, groups, data_format)


@_amp_op('conv3d')
def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format='NCDHW',
           name=None):
    return _conv(TF.conv3d, 3, x, weight, bias, stride, padding, dilation, groups, data_format)


def _conv_t(fn, n, x, weight, bias, stride, padding, output_padding, dilation, groups, output_size,
            data_format):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC')
    if cl:
        t = t.movedim(-1, 1)
    pad_, _ = _conv_padding(padding, n)
    if pad_ == 'same':
        pad_ = tuple((k - 1) // 2 for k in _t(weight).shape[2:])
    st, dl = _ntuple(stride, n), _ntuple(dilation, n)
    op = _ntuple(output_padding, n)
    if output_size is not None:
        if isinstance(output_size, int):
            output_size = [output_size] * n
        ks = _t(weight).shape[2:]
        base = [(t.shape[2 + i] - 1) * st[i] - 2 * pad_[i] + dl[i] * (ks[i] - 1) + 1 for i in range(n)]
        op = tuple(int(o) - b for o, b in zip(output_size, base))
    out = fn(t, _t(weight), None if bias is None else _t(bias), st, pad_, op, groups, dl)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                     dilation=1, output_size=None, data_format='NCL', name=None):
    return _conv_t(TF.conv_transpose1d, 1, x, weight, bias, stride, padding, output_padding, dilation,
                   groups, output_size, data_format)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, dilation=1,
                     groups=1, output_size=None, data_format='NCHW', name=None):
    return _conv_t(TF.conv_transpose2d, 2, x, weight, bias, stride, padding, output_padding, dilation,
                   groups, output_size, data_format)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                     dilation=1, output_size=None, data_format='NCDHW', name=None):
    return _conv_t(TF.conv_transpose3d, 3, x, weight, bias, stride, padding, output_padding, dilation,
                   groups, output_size, data_format)


def _pool_pad(padding, n):
    if isinstance(padding, str):
        return padding.upper(), None
    if isinstance(padding, (list, tuple)) and len(padding) == 2 * n:
        if all(padding[2 * i] == padding[2 * i + 1] for i in range(n)):
            return tuple(padding[0::2]), None
        tp = []
        for i in reversed(range(n)):
            tp += [padding[2 * i], padding[2 * i + 1]]
        return 0, tp
    return _ntuple(padding, n), None


def _pool(kind, n, x, kernel_size, stride, padding, ceil_mode, data_format, exclusive=True,
          return_mask=False, divisor_override=None):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC')
    if kind == 'max' and n == 2 and cl and not ceil_mode and not return_mask and t.is_cuda:
        ks = _ntuple(kernel_size, 2)
        st = ks if stride is None else _ntuple(stride, 2)
        pd, extra = _pool_pad(padding, 2)
        if extra is None and not isinstance(pd, str) and K.max_pool_nhwc_supported(t, ks, st, pd):
            return _w(K.max_pool2d_nhwc(t, ks, st, pd))
    if cl:
        t = t.movedim(-1, 1)
    ks = _ntuple(kernel_size, n)
    st = ks if stride is None else _ntuple(stride, n)
    pd, extra = _pool_pad(padding, n)
    if pd == 'VALID':
        pd = (0,) * n
    elif pd == 'SAME':
        outs = [math.ceil(t.shape[2 + i] / st[i]) for i in range(n)]
        tot = [max((outs[i] - 1) * st[i] + ks[i] - t.shape[2 + i], 0) for i in range(n)]
        extra = []
        for i in reversed(range(n)):
            extra += [tot[i] // 2, tot[i] - tot[i] // 2]
        pd = (0,) * n
    if extra is not None:
        t = TF.pad(t, extra, value=float('-inf') if kind == 'max' else 0.0)
    if kind == 'max':
        fn = {1: TF.max_pool1d, 2: TF.max_pool2d, 3: TF.max_pool3d}[n]
        r = fn(t, ks, st, pd, 1, ceil_mode, return_mask)
        if return_mask:
            out, mask = r
            return (_w(out.movedim(1, -1) if cl else out), _w(mask))
        out = r
    else:
        fn = {1: TF.avg_pool1d, 2: TF.avg_pool2d, 3: TF.avg_pool3d}[n]
        kw = {} if n == 1 else {'divisor_override': divisor_override}
        out = fn(t, ks, st, pd, ceil_mode, not exclusive, **kw)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
               name=None):
    return _pool('max', 1, x, kernel_size, stride, padding, ceil_mode, 'NCL', return_mask=return_mask)


def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
               data_format='NCHW', name=None):
    return _pool('max', 2, x, kernel_size, stride, padding, ceil_mode, data_format,
                 return_mask=return_mask)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
               data_format='NCDHW', name=None):
    return _pool('max', 3, x, kernel_size, stride, padding, ceil_mode, data_format,
                 return_mask=return_mask)


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    return _pool('avg', 1, x, kernel_size, stride, padding, ceil_mode, 'NCL', exclusive)


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
               divisor_override=None, data_format='NCHW', name=None):
    return _pool('avg', 2, x, kernel_size, stride, padding, ceil_mode, data_format, exclusive,
                 divisor_override=divisor_override)


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True,
               divisor_override=None, data_format='NCDHW', name=None):
    return _pool('avg', 3, x, kernel_size, stride, padding, ceil_mode, data_format, exclusive,
                 divisor_override=divisor_override)


def _adaptive(fn, x, output_size, data_format, return_mask=False):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC')
    if cl:
        t = t.movedim(-1, 1)
    if isinstance(output_size, (list, tuple)):
        output_size = tuple(t.shape[2 + i] if o is None else o for i, o in enumerate(output_size))
    r = fn(t, output_size, return_mask) if return_mask else fn(t, output_size)
    if return_mask:
        return _w(r[0]), _w(r[1])
    return _w(r.movedim(1, -1) if cl else r)


def adaptive_avg_pool1d(x, output_size, name=None):
    return _adaptive(TF.adaptive_avg_pool1d, x, output_size, 'NCL')


def adaptive_avg_pool2d(x, output_size, data_format='NCHW', name=None):
    if data_format == 'NHWC' and output_size in (1, (1, 1), [1, 1]):
        t = _t(x)
        if K.global_avg_pool_nhwc_supported(t):
            return _w(K.GlobalAvgPoolNHWCFn.apply(t))
    return _adaptive(TF.adaptive_avg_pool2d, x, output_size, data_format)


def adaptive_avg_pool3d(x, output_size, data_format='NCDHW', name=None):
    return _adaptive(TF.adaptive_avg_pool3d, x, output_size, data_format)


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    return _adaptive(TF.adaptive_max_pool1d, x, output_size, 'NCL', return_mask)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    return _adaptive(TF.adaptive_max_pool2d, x, output_size, 'NCHW', return_mask)


def adaptive_max_pool3d(x, output_size, return_mask=False, name=None):
    return _adaptive(TF.adaptive_max_pool3d, x, output_size, 'NCDHW', return_mask)


def max_unpool1d(x, indices, kernel_size, stride=None, padding=0, data_format='NCL',
                 output_size=None, name=None):
    return _w(TF.max_unpool1d(_t(x), _t(indices), kernel_size, stride, padding, output_size))


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, data_format='NCHW',
                 output_size=None, name=None):
    return _w(TF.max_unpool2d(_t(x), _t(indices), kernel_size, stride, padding, output_size))


def max_unpool3d(x, indices, kernel_size, stride=None, padding=0, data_format='NCDHW',
                 output_size=None, name=None):
    return _w(TF.max_unpool3d(_t(x), _t(indices), kernel_size, stride, padding, output_size))


# =============================================================================
# norms
# =============================================================================
@_amp_op('layer_norm')
def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-05, name=None):
    t = _t(x)
    if isinstance(normalized_shape, int):
        normalized_shape = [normalized_shape]
    w, b = _opt(weight), _opt(bias)
    n = int(np.prod(normalized_shape))
    if w is not None and w.dim() > 1:
        w = w.reshape(-1)
    if b is not None and b.dim() > 1:
        b = b.reshape(-1)
    if t.dtype in (torch.float32, torch.float16, torch.bfloat16) and (w is None or w.numel() == n):
        shp = t.shape
        out = K.layer_norm(t.reshape(*shp[:t.dim() - len(normalized_shape)], n), w, b, epsilon)
        return _w(out.reshape(shp))
    return _w(TF.layer_norm(t, list(normalized_shape), w, b, epsilon))


def rms_norm(x, weight=None, epsilon=1e-6, name=None):
    return _w(K.rms_norm(_t(x), _opt(weight), epsilon))


@_amp_op('batch_norm')
def batch_norm(x, running_mean, running_var, weight, bias, training=False, momentum=0.9,
               epsilon=1e-05, data_format='NCHW', use_global_stats=None, name=None):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC') or t.dim() == 2
    if use_global_stats:
        training = False
    rm, rv = _t(running_mean), _t(running_var)
    if cl and t.is_cuda and t.shape[-1] % 8 == 0 and rm.dtype == torch.float32:
        # channels-last on the device: gfx950 BN kernel (ops/csrc/bn.hip)
        return _w(K.batch_norm_act(t, None, _opt(weight), _opt(bias), rm, rv, training,
                                   momentum, epsilon, False))
    if cl:
        t = t.movedim(-1, 1)
    w = _opt(weight)
    if rm.dtype != t.dtype and not (w is not None and w.dtype == torch.float32):
        rm, rv = rm.to(t.dtype), rv.to(t.dtype)  # (mixed bf16-in/fp32-param runs natively)
    out = TF.batch_norm(t, rm, rv, w, _opt(bias), training, 1 - momentum, epsilon)
    if cl:
        out = out.movedim(1, -1)
    return _w(out)


def fused_bn_add_act(x, z, running_mean, running_var, weight, bias, training=False, momentum=0.9,
                     epsilon=1e-05, act='relu', data_format='NHWC'):
    """act(batch_norm(x) + z) in one pass (parity: fluid/operators/fused/
    fused_bn_add_activation_op.cu; ``z=None`` is fused_bn_activation). Channels-last on the
    device runs the gfx950 kernel; other layouts compose."""
    if act not in (None, 'relu', 'identity'):
        raise ValueError(f"fused_bn_add_act: unsupported act {act!r}")
    relu = act == 'relu'
    t = _t(x)
    rm, rv = _t(running_mean), _t(running_var)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC') or t.dim() == 2
    if cl and rm.dtype == torch.float32 and (t.shape[-1] % 8 == 0 or not t.is_cuda):
        return _w(K.batch_norm_act(t, _opt(z), _opt(weight), _opt(bias), rm, rv, training,
                                   momentum, epsilon, relu))
    out = _t(batch_norm(x, running_mean, running_var, weight, bias, training, momentum, epsilon,
                        data_format))
    if z is not None:
        out = out + _t(z)
    return _w(torch.relu(out) if relu else out)


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None,
                  use_input_stats=True, momentum=0.9, eps=1e-05, data_format='NCHW', name=None):
    return _w(TF.instance_norm(_t(x), _opt(running_mean), _opt(running_var), _opt(weight), _opt(bias),
                               use_input_stats, 1 - momentum, eps))


def group_norm(x, num_groups, epsilon=1e-05, weight=None, bias=None, data_format='NCHW', name=None):
    t = _t(x)
    cl = data_format in ('NHWC', 'NLC', 'NDHWC')
    if cl:
        t = t.movedim(-1, 1)
    out = TF.group_norm(t, num_groups, _opt(weight), _opt(bias), epsilon)
    return _w(out.movedim(1, -1) if cl else out)


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0, data_format='NCHW', name=None):
    return _w(TF.local_response_norm(_t(x), size, alpha * size, beta, k))


# =============================================================================
# losses
# =============================================================================
def _reduce(loss, reduction):
    if reduction == 'mean':
        return loss.mean()
    if reduction == 'sum':
        return loss.sum()
    return loss


@_amp_op('cross_entropy')
def cross_entropy(input, label, weight=None, ignore_index=-100, reduction='mean', soft_label=False,
                  axis=-1, use_softmax=True, label_smoothing=0.0, name=None):
    """Paddle cross_entropy. Hard labels on the HIP device use the fused
    one-pass softmax+CE kernel (the [N, V] probabilities are never stored)."""
    x, lab = _t(input), _t(label)
    nd = x.dim()
    axis = axis % nd
    if not use_softmax:
        logp = torch.log(x.clamp_min(1e-30))
        if soft_label:
            loss = -(lab * logp).sum(axis)
        else:
            l = lab.squeeze(axis) if lab.dim() == nd else lab
            loss = TF.nll_loss(logp.movedim(axis, 1) if nd > 2 else logp, l.long(),
                               None if weight is None else _t(weight), reduction='none',
                               ignore_index=ignore_index)
        return _w(_reduce(loss, reduction))
    if soft_label or (lab.dtype.is_floating_point and lab.shape == x.shape):
        logp = torch.log_softmax(x.float(), axis)
        loss = -(lab.float() * logp).sum(axis)
        if weight is not None:
            loss = loss * (lab.float() * _t(weight)).sum(axis)
        return _w(_reduce(loss, reduction).to(x.dtype if x.dtype != torch.bfloat16 else torch.float32))
    l = lab.squeeze(axis) if (lab.dim() == nd and lab.shape[axis] == 1) else lab
    l = l.long()
    if (axis == nd - 1 and weight is None and label_smoothing == 0.0 and
            x.dtype in (torch.float32, torch.float16, torch.bfloat16)):
        loss = K.softmax_cross_entropy(x, l, ignore_index)
        if reduction == 'mean':
            valid = (l != ignore_index).sum().clamp_min(1)
            return _w(loss.sum() / valid)
        return _w(_reduce(loss, reduction))
    xm = x.movedim(axis, 1) if nd > 2 else x
    loss = TF.cross_entropy(xm.float(), l, None if weight is None else _t(weight).float(),
                            ignore_index=ignore_index, reduction=reduction,
                            label_smoothing=label_smoothing)
    return _w(loss)


@_amp_op('softmax_with_cross_entropy')
def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100,
                               numeric_stable_mode=True, return_softmax=False, axis=-1):
    x, lab = _t(logits), _t(label)
    nd = x.dim()
    axis = axis % nd
    if soft_label:
        loss = -(lab * torch.log_softmax(x, axis)).sum(axis, keepdim=True)
    else:
        l = lab.squeeze(axis) if lab.dim() == nd else lab
        if axis == nd - 1 and x.dtype in (torch.float32, torch.float16, torch.bfloat16):
            loss = K.softmax_cross_entropy(x, l.long(), ignore_index).unsqueeze(axis)
        else:
            loss = TF.cross_entropy(x.movedim(axis, 1), l.long(), ignore_index=ignore_index,
                                    reduction='none').unsqueeze(axis)
    if return_softmax:
        return _w(loss), _w(torch.softmax(x, axis))
    return _w(loss)


def nll_loss(input, label, weight=None, ignore_index=-100, reduction='mean', name=None):
    return _w(TF.nll_loss(_t(input), _t(label).long(), _opt(weight), ignore_index=ignore_index,
                          reduction=reduction))


@_amp_op('mse_loss')
def mse_loss(input, label, reduction='mean', name=None):
    return _w(TF.mse_loss(_t(input), _t(label), reduction=reduction))


def square_error_cost(input, label):
    return _w((_t(input) - _t(label)) ** 2)


def l1_loss(input, label, reduction='mean', name=None):
    return _w(TF.l1_loss(_t(input), _t(label), reduction=reduction))


def smooth_l1_loss(input, label, reduction='mean', delta=1.0, name=None):
    return _w(TF.huber_loss(_t(input), _t(label), reduction=reduction, delta=delta))


def binary_cross_entropy(input, label, weight=None, reduction='mean', name=None):
    return _w(TF.binary_cross_entropy(_t(input), _t(label), _opt(weight), reduction=reduction))


def binary_cross_entropy_with_logits(logit, label, weight=None, reduction='mean', pos_weight=None,
                                     name=None):
    return _w(TF.binary_cross_entropy_with_logits(_t(logit), _t(label), _opt(weight),
                                                  reduction=reduction, pos_weight=_opt(pos_weight)))


def kl_div(input, label, reduction='mean', name=None):
    t, l = _t(input), _t(label)
    loss = l * (torch.log(l.clamp_min(1e-30)) - t)
    loss = torch.where(l > 0, loss, torch.zeros_like(loss))
    if reduction == 'batchmean':
        return _w(loss.sum() / t.shape[0])
    return _w(_reduce(loss, reduction))


def margin_ranking_loss(input, other, label, margin=0.0, reduction='mean', name=None):
    return _w(TF.margin_ranking_loss(_t(input), _t(other), _t(label), margin, reduction=reduction))


def hinge_embedding_loss(input, label, margin=1.0, reduction='mean', name=None):
    return _w(TF.hinge_embedding_loss(_t(input), _t(label), margin, reduction=reduction))


def cosine_embedding_loss(input1, input2, label, margin=0, reduction='mean', name=None):
    return _w(TF.cosine_embedding_loss(_t(input1), _t(input2), _t(label), margin, reduction=reduction))


def soft_margin_loss(input, label, reduction='mean', name=None):
    return _w(TF.soft_margin_loss(_t(input), _t(label).to(_t(input).dtype), reduction=reduction))


def multi_label_soft_margin_loss(input, label, weight=None, reduction='mean', name=None):
    return _w(TF.multilabel_soft_margin_loss(_t(input), _t(label), _opt(weight), reduction=reduction))


def multi_margin_loss(input, label, p=1, margin=1.0, weight=None, reduction='mean', name=None):
    return _w(TF.multi_margin_loss(_t(input), _t(label).long(), p, margin, _opt(weight),
                                   reduction=reduction))


def triplet_margin_loss(input, positive, negative, margin=1.0, p=2, epsilon=1e-6, swap=False,
                        reduction='mean', name=None):
    return _w(TF.triplet_margin_loss(_t(input), _t(positive), _t(negative), margin, p, epsilon, swap,
                                     reduction=reduction))


def triplet_margin_with_distance_loss(input, positive, negative, distance_function=None, margin=1.0,
                                      swap=False, reduction='mean', name=None):
    df = None
    if distance_function is not None:
        df = lambda a, b: _t(distance_function(Tensor(a), Tensor(b)))
    return _w(TF.triplet_margin_with_distance_loss(_t(input), _t(positive), _t(negative),
                                                   distance_function=df, margin=margin, swap=swap,
                                                   reduction=reduction))


def log_loss(input, label, epsilon=1e-4, name=None):
    t, l = _t(input), _t(label)
    return _w(-l * torch.log(t + epsilon) - (1 - l) * torch.log(1 - t + epsilon))


def sigmoid_focal_loss(logit, label, normalizer=None, alpha=0.25, gamma=2.0, reduction='sum',
                       name=None):
    x, l = _t(logit), _t(label)
    p = torch.sigmoid(x)
    ce = TF.binary_cross_entropy_with_logits(x, l, reduction='none')
    pt = p * l + (1 - p) * (1 - l)
    loss = ce * ((1 - pt) ** gamma)
    if alpha >= 0:
        loss = (alpha * l + (1 - alpha) * (1 - l)) * loss
    if normalizer is not None:
        loss = loss / _t(normalizer)
    return _w(_reduce(loss, reduction))


def dice_loss(input, label, epsilon=0.00001, name=None):
    x = _t(input)
    l = TF.one_hot(_t(label).long().squeeze(-1), x.shape[-1]).to(x.dtype)
    red = tuple(range(1, x.dim()))
    inter = (x * l).sum(red)
    return _w((1 - 2 * inter / (x.sum(red) + l.sum(red) + epsilon)).mean())


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    a, p, l = _t(anchor), _t(positive), _t(labels).float().reshape(-1, 1)
    same = (l == l.t()).float()
    same = same / same.sum(1, keepdim=True)
    logits = a @ p.t()
    ce = (-same * torch.log_softmax(logits, 1)).sum(1).mean()
    reg = l2_reg * ((a ** 2).sum(1).mean() + (p ** 2).sum(1).mean()) * 0.25
    return _w(ce + reg)


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction='mean',
             norm_by_times=False):
    loss = TF.ctc_loss(_t(log_probs), _t(labels), _t(input_lengths), _t(label_lengths), blank,
                       reduction='none')
    if reduction == 'mean':
        return _w((loss / _t(label_lengths).clamp_min(1)).mean())
    return _w(_reduce(loss, reduction))


def rnnt_loss(input, label, input_lengths, label_lengths, blank=0, fastemit_lambda=0.001,
              reduction='mean', name=None):
    """RNN-Transducer loss (parity: python/paddle/nn/functional/loss.py:1818 rnnt_loss over
    warp-transducer). ``input`` [B, T, U+1, V] are unnormalised joint-network outputs
    (log-softmax is applied here, as the reference's GPU path does).

    Forward variable in log space, one vectorised update per time step: within a row t the
    label recursion alpha[t,u] = logaddexp(alpha[t-1,u] + blank[t-1,u], alpha[t,u-1] +
    emit[t,u-1]) is a linear recurrence, solved as E[u] + logcumsumexp(a[u] - E[u]) with E
    the running sum of emission log-probs — T batched kernels instead of T*U scalar steps.
    Gradients come from autograd through the recursion. FastEmit (arXiv 2010.11148) scales
    the emission-path gradient by (1 + lambda) and leaves the loss value unchanged."""
    x = _t(input)
    lab = _t(label).long()
    tl, ul = _t(input_lengths).long().to(x.device), _t(label_lengths).long().to(x.device)
    B, T, U1, V = x.shape
    lp = torch.log_softmax(x.float() if x.dtype in (torch.float16, torch.bfloat16) else x, -1)
    blank_lp = lp[..., blank]                                            # [B, T, U+1]
    U = U1 - 1
    if U > 0:
        emit = torch.gather(lp[:, :, :U, :], 3,
                            lab[:, None, :U, None].expand(B, T, U, 1).clamp_min(0)).squeeze(-1)
    else:
        emit = lp.new_zeros(B, T, 0)
    if fastemit_lambda:
        emit = emit + fastemit_lambda * (emit - emit.detach())
    ninf = torch.finfo(lp.dtype).min / 4
    E = torch.cat([emit.new_zeros(B, T, 1), torch.cumsum(emit, -1)], -1)  # [B, T, U+1]
    alphas = []
    a = torch.full((B, U1), ninf, dtype=lp.dtype, device=lp.device)
    a[:, 0] = 0.0
    for t in range(T):
        if t > 0:
            a = alphas[-1] + blank_lp[:, t - 1]
        alpha = E[:, t] + torch.logcumsumexp(a - E[:, t], -1)
        alphas.append(alpha)
    alpha = torch.stack(alphas, 1)                                        # [B, T, U+1]
    bi = torch.arange(B, device=lp.device)
    tT = (tl - 1).clamp_min(0)
    loss = -(alpha[bi, tT, ul] + blank_lp[bi, tT, ul])
    if reduction == 'mean':
        return _w(loss.sum() / B)
    if reduction == 'sum':
        return _w(loss.sum())
    return _w(loss)


def _hs_default_paths(lab, num_classes):
    """Default complete-binary-tree codes (matrix_bit_code.h SimpleCode): code = label +
    num_classes; step j visits node (code >> (j+1)) - 1 with target bit (code >> j) & 1."""
    L = max(int(num_classes - 1).bit_length(), 1)
    code = lab + num_classes
    j = torch.arange(L, device=lab.device)
    node = (code[:, None] >> (j + 1)) - 1
    bit = (code[:, None] >> j) & 1
    valid = node >= 0
    return node, bit, valid


def hsigmoid_loss(input, label, num_classes, weight, bias=None, path_table=None,
                  path_code=None, is_sparse=False, name=None):
    """Hierarchical sigmoid (parity: python/paddle/nn/functional/loss.py hsigmoid_loss over
    phi hierarchical_sigmoid kernel). Returns [N, 1]: per sample the sum over its tree path
    of softplus(pre) - bit * pre, pre = clip(x . W[node] + b[node], -40, 40). Like the
    reference kernel, padded path slots (shorter paths of the default tree) contribute
    softplus(0) = log 2 each; custom trees pass ``path_table``/``path_code`` ([N, L], -1
    terminated). One batched gather + contraction, no per-sample loop."""
    x = _t(input)
    lab = _t(label).long().reshape(-1)
    W = _t(weight)
    if path_table is not None:
        node = _t(path_table).long()
        bit = _t(path_code).long()
        valid = torch.cumprod((node >= 0).long(), -1).bool()
    else:
        node, bit, valid = _hs_default_paths(lab, num_classes)
    safe = node.clamp_min(0)
    pre = torch.einsum('nd,nld->nl', x, W[safe])
    if bias is not None:
        pre = pre + _t(bias).reshape(-1)[safe]
    pre = torch.where(valid, pre, torch.zeros_like(pre)).clamp(-40.0, 40.0)
    out = TF.softplus(pre).sum(-1) - (pre * (bit * valid).to(pre.dtype)).sum(-1)
    return _w(out.unsqueeze(-1))


def margin_cross_entropy(logits, label, margin1=1.0, margin2=0.5, margin3=0.0, scale=64.0,
                         group=None, return_softmax=False, reduction='mean'):
    x, l = _t(logits), _t(label).long().reshape(-1)
    theta = torch.acos(x.clamp(-1, 1))
    tgt = torch.cos(margin1 * theta + margin2) - margin3
    oh = TF.one_hot(l, x.shape[-1]).bool()
    z = torch.where(oh, tgt, x) * scale
    loss = TF.cross_entropy(z, l, reduction='none').unsqueeze(-1)
    loss = _reduce(loss, reduction) if reduction else loss
    if return_softmax:
        return _w(loss), _w(torch.softmax(z, -1))
    return _w(loss)


# =============================================================================
# attention
# =============================================================================
def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False,
                                 training=True, name=None):
    """Inputs [batch, seq, heads, head_dim] (paddle layout)."""
    q, k, v = _t(query), _t(key), _t(value)
    drop = dropout_p if training else 0.0
    if attn_mask is None and drop == 0.0 and q.is_cuda:
        return _w(K.flash_attention(q, k, v, causal=is_causal))
    # additive / boolean mask and dropout: the flash kernel's extended path on the device (fp32
    # reference of the same math, same dropout bits, on the host)
    return _w(K.flash_attention_ext(q, k, v, causal=is_causal, attn_mask=_opt(attn_mask),
                                    dropout=drop))


def _seed_of(fixed_seed_offset):
    if fixed_seed_offset is None:
        return None
    so = _t(fixed_seed_offset).reshape(-1).tolist()
    return int(so[0])


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False,
                    fixed_seed_offset=None, rng_name="", training=True, name=None):
    """paddle.nn.functional.flash_attention.flash_attention -> (out, softmax|None) (parity:
    python/paddle/nn/functional/flash_attention.py:20). Dropout runs inside the flash kernel.
    ``return_softmax`` (a debugging output of the reference) returns the dropped probabilities
    from the fp32 reference of the same kernel math."""
    q, k, v = _t(query), _t(key), _t(value)
    drop = dropout if training else 0.0
    if drop > 0:
        out = _w(K.flash_attention_ext(q, k, v, causal=causal, dropout=drop,
                                       seed=_seed_of(fixed_seed_offset)))
    else:
        out = _w(K.flash_attention(q, k, v, causal=causal))
    sm = None
    if return_softmax:
        with torch.no_grad():
            B, Sq, H, D = q.shape
            qf, kf = q.float().permute(0, 2, 1, 3), k.float().permute(0, 2, 1, 3)
            s_ = torch.matmul(qf, kf.transpose(-1, -2)) / math.sqrt(D)
            if causal:
                Sk = kf.shape[2]
                s_ = s_.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(Sk - Sq + 1),
                                    float('-inf'))
            sm = _w(torch.softmax(s_, -1).to(q.dtype))
    return out, sm


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                        scale, dropout=0.0, causal=False, return_softmax=False,
                        fixed_seed_offset=None, rng_name="", training=True, name=None):
    """Variable-length (packed) flash attention (parity: python/paddle/nn/functional/
    flash_attention.py:121 flash_attn_unpadded): query [total_q, H, D], key/value
    [total_k, H, D], cu_seqlens_* int32 [B+1]; one HIP launch covers every sequence."""
    q, k, v = _t(query), _t(key), _t(value)
    out = K.flash_attn_varlen(q, k, v, _t(cu_seqlens_q), _t(cu_seqlens_k), int(max_seqlen_q),
                              int(max_seqlen_k), causal=causal, scale=float(scale),
                              dropout=dropout if training else 0.0, seed=_seed_of(fixed_seed_offset))
    return _w(out), None


def sparse_attention(query, key, value, sparse_csr_offset, sparse_csr_columns,
                     key_padding_mask=None, attn_mask=None, name=None):
    """softmax(Q·Kᵀ/√d restricted to a CSR layout) · V (parity:
    python/paddle/nn/functional/sparse_attention.py). The per-(batch, head) CSR pattern
    [S+1 offsets, nnz columns] is scattered into a boolean layout once; key_padding_mask
    [B, S] and attn_mask [S, S] (0 = masked) narrow it further. Rows with no admitted key
    return zeros."""
    q, k, v = _t(query), _t(key), _t(value)
    b, h, s, d = q.shape
    off = _t(sparse_csr_offset).long().reshape(b * h, s + 1)
    cols = _t(sparse_csr_columns).long().reshape(b * h, -1)
    nnz = cols.shape[1]
    row = torch.searchsorted(off[:, 1:].contiguous(),
                             torch.arange(nnz, device=q.device).expand(b * h, nnz).contiguous(),
                             right=True)
    valid = torch.arange(nnz, device=q.device)[None] < off[:, -1:]
    layout = torch.zeros(b * h, s, s, dtype=torch.bool, device=q.device)
    bh = torch.arange(b * h, device=q.device)[:, None].expand_as(row)
    layout[bh[valid], row.clamp(max=s - 1)[valid], cols[valid]] = True
    layout = layout.view(b, h, s, s)
    if key_padding_mask is not None:
        layout = layout & (_t(key_padding_mask) != 0).view(b, 1, 1, s)
    if attn_mask is not None:
        layout = layout & (_t(attn_mask) != 0).view(1, 1, s, s)
    sc = torch.matmul(q.float(), k.float().transpose(-1, -2)) / math.sqrt(d)
    sc = sc.masked_fill(~layout, float('-inf'))
    p = torch.softmax(sc, -1).nan_to_num(0.0)
    return _w(torch.matmul(p, v.float()).to(q.dtype))


def class_center_sample(label, num_classes, num_samples, group=None):
    l = _t(label).reshape(-1)
    pos = torch.unique(l)
    if pos.numel() < num_samples:
        others = torch.tensor([i for i in range(num_classes) if i not in set(pos.tolist())],
                              device=l.device)
        perm = others[torch.randperm(others.numel(), device=l.device)[:num_samples - pos.numel()]]
        sampled = torch.cat([pos, perm]).sort().values
    else:
        sampled = pos
    remap = torch.full((num_classes,), -1, dtype=torch.long, device=l.device)
    remap[sampled] = torch.arange(sampled.numel(), device=l.device)
    return _w(remap[l]), _w(sampled)


def gather_tree(ids, parents):
    i, p = _t(ids), _t(parents)
    T = i.shape[0]
    out = torch.empty_like(i)
    out[-1] = i[-1]
    par = p[-1]
    for t in range(T - 2, -1, -1):
        out[t] = torch.gather(i[t], -1, par)
        par = torch.gather(p[t], -1, par)
    return _w(out)
