"""paddle.static.nn (parity: python/paddle/static/nn/common.py): layer-building functions
usable in static programs (parameters created eagerly, ops recorded)."""
from .. import nn as _nn
from ..nn import functional as F
from ..framework.core import Tensor, _u

_layers = []  # keep created layers alive (their params are referenced by the program)


def _keep(l):
    _layers.append(l)
    return l


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    in_f = 1
    for s in x.shape[num_flatten_dims:]:
        in_f *= s
    lin = _keep(_nn.Linear(in_f, size, weight_attr, bias_attr))
    if len(x.shape) > num_flatten_dims + 1:
        x = x.flatten(num_flatten_dims)
    out = lin(x)
    if activation:
        out = getattr(F, activation)(out)
    return out


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None,
              param_attr=None, dtype='float32'):
    return _keep(_nn.Embedding(size[0], size[1], padding_idx, weight_attr=param_attr))(input)


sparse_embedding = embedding


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
           param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
           data_format="NCHW"):
    cin = input.shape[1] if data_format == 'NCHW' else input.shape[-1]
    out = _keep(_nn.Conv2D(cin, num_filters, filter_size, stride, padding, dilation, groups or 1,
                           weight_attr=param_attr, bias_attr=bias_attr,
                           data_format=data_format))(input)
    return getattr(F, act)(out) if act else out


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0,
                     stride=1, dilation=1, groups=None, param_attr=None, bias_attr=None,
                     use_cudnn=True, act=None, name=None, data_format='NCHW'):
    cin = input.shape[1]
    out = _keep(_nn.Conv2DTranspose(cin, num_filters, filter_size, stride, padding,
                                    dilation=dilation, groups=groups or 1,
                                    weight_attr=param_attr, bias_attr=bias_attr))(input)
    return getattr(F, act)(out) if act else out


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
           param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
           data_format="NCDHW"):
    out = _keep(_nn.Conv3D(input.shape[1], num_filters, filter_size, stride, padding, dilation,
                           groups or 1, weight_attr=param_attr, bias_attr=bias_attr))(input)
    return getattr(F, act)(out) if act else out


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0,
                     stride=1, dilation=1, groups=None, param_attr=None, bias_attr=None,
                     use_cudnn=True, act=None, name=None, data_format='NCDHW'):
    out = _keep(_nn.Conv3DTranspose(input.shape[1], num_filters, filter_size, stride,
                                    padding))(input)
    return getattr(F, act)(out) if act else out


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None,
               bias_attr=None, data_layout='NCHW', in_place=False, name=None,
               moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=True, use_global_stats=False):
    c = input.shape[1] if data_layout == 'NCHW' else input.shape[-1]
    bn = _keep(_nn.BatchNorm(c, act, is_test, momentum, epsilon, param_attr, bias_attr,
                             data_layout=data_layout, use_global_stats=use_global_stats))
    return bn(input)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None,
               bias_attr=None, act=None, name=None):
    shp = input.shape[begin_norm_axis:]
    out = _keep(_nn.LayerNorm(shp, epsilon, param_attr if scale else False,
                              bias_attr if shift else False))(input)
    return getattr(F, act)(out) if act else out


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None,
               data_layout='NCHW', name=None):
    out = _keep(_nn.GroupNorm(groups, input.shape[1], epsilon, param_attr, bias_attr))(input)
    return getattr(F, act)(out) if act else out


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):
    return _keep(_nn.InstanceNorm2D(input.shape[1], epsilon))(input)


def prelu(x, mode='all', param_attr=None, data_format="NCHW", name=None):
    n = 1 if mode == 'all' else x.shape[1]
    return _keep(_nn.PReLU(n, weight_attr=param_attr, data_format=data_format))(x)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    out = _keep(_nn.Bilinear(x.shape[-1], y.shape[-1], size, param_attr, bias_attr))(x, y)
    return getattr(F, act)(out) if act else out


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    return _keep(_nn.SpectralNorm(weight.shape, dim, power_iters, eps))(weight)


class _DataNorm(_nn.Layer):
    """data_norm (parity: paddle/fluid/operators/data_norm_op.cc): normalise with ACCUMULATED
    batch statistics — y = (x - BatchSum/BatchSize) * sqrt(BatchSize/BatchSquareSum) — not
    the current batch's. In training the statistics absorb each batch with the summary decay
    (size += N, sum += Σx, square_sum += Σ(x-mean)^2 + N·eps, all decayed first)."""

    def __init__(self, C, epsilon, param_attr, slot_dim, decay, scale_shift):
        super().__init__()
        from ..nn import initializer as I
        pa = param_attr if isinstance(param_attr, dict) else {}
        self.batch_size = self.create_parameter(
            [C], default_initializer=I.Constant(pa.get('batch_size', 1e4)))
        self.batch_sum = self.create_parameter(
            [C], default_initializer=I.Constant(pa.get('batch_sum', 0.0)))
        self.batch_square_sum = self.create_parameter(
            [C], default_initializer=I.Constant(pa.get('batch_square', 1e4)))
        for p in (self.batch_size, self.batch_sum, self.batch_square_sum):
            p.stop_gradient = True
        self.scale_w = self.create_parameter([C], default_initializer=I.Constant(1.0)) \
            if scale_shift else None
        self.bias = self.create_parameter([C], is_bias=True) if scale_shift else None
        self.eps, self.slot_dim, self.decay = epsilon, slot_dim, decay

    def forward(self, x):
        import torch
        t = _u(x)
        bs, su, sq = self.batch_size._t, self.batch_sum._t, self.batch_square_sum._t
        mean = su / bs
        scale = torch.sqrt(bs / sq)
        y = (t - mean) * scale
        if self.slot_dim > 0:  # slots whose show count (first column) is 0 stay zero
            n = t.shape[-1] // self.slot_dim
            show = t.reshape(*t.shape[:-1], n, self.slot_dim)[..., :1]
            y = (y.reshape(*t.shape[:-1], n, self.slot_dim) * (show > 0)).reshape(t.shape)
        if self.scale_w is not None:
            y = y * self.scale_w._t + self.bias._t
        if self.training:
            with torch.no_grad():
                x2 = t.detach().reshape(-1, t.shape[-1])
                N = x2.shape[0]
                bs.mul_(self.decay).add_(N)
                su.mul_(self.decay).add_(x2.sum(0))
                sq.mul_(self.decay).add_(((x2 - mean) ** 2).sum(0) + N * self.eps)
        return Tensor(y)


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout='NCHW',
              in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
              do_model_average_for_mean_and_var=True, slot_dim=-1, sync_stats=False,
              summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    out = _keep(_DataNorm(input.shape[-1], epsilon, param_attr, slot_dim, summary_decay_rate,
                          enable_scale_and_shift))(input)
    return getattr(F, act)(out) if act else out


def deform_conv2d(x, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1,
                  groups=1, deformable_groups=1, im2col_step=1, weight_attr=None, bias_attr=None,
                  name=None):
    """Deformable conv v1 (mask None) / v2 (parity: static/nn/common.py deform_conv2d) on
    paddle_ray_amd.vision.ops.DeformConv2D."""
    from ..vision.ops import DeformConv2D
    layer = _keep(DeformConv2D(x.shape[1], num_filters, filter_size, stride, padding, dilation,
                               deformable_groups, groups, weight_attr, bias_attr))
    return layer(x, offset, mask)


class _NCE(_nn.Layer):
    """Noise-contrastive estimation (parity: paddle/fluid/operators/nce_op.h): for the true
    class and ``num_neg_samples`` sampled classes, o = sigmoid(x.w_c + b_c) and
    b = k * q(c); cost = -log(o / (o + b)) (true) - Σ log(b / (o + b)) (sampled)."""

    def __init__(self, dim, num_classes, num_neg, sampler, custom_dist, seed, param_attr,
                 bias_attr):
        super().__init__()
        self.weight = self.create_parameter([num_classes, dim], param_attr)
        self.bias = self.create_parameter([num_classes, 1], bias_attr, is_bias=True) \
            if bias_attr is not False else None
        self.C, self.k, self.sampler = num_classes, num_neg, sampler
        self.custom = None if custom_dist is None else list(custom_dist)
        self.gen = None
        if seed:
            import torch
            self.gen = torch.Generator().manual_seed(int(seed))

    def _q(self, c):
        import torch
        if self.sampler == 'uniform':
            return torch.full(c.shape, 1.0 / self.C, dtype=torch.float32, device=c.device)
        if self.sampler == 'log_uniform':
            cf = c.float()
            return torch.log((cf + 2) / (cf + 1)) / torch.log(torch.tensor(self.C + 1.0))
        dist = torch.tensor(self.custom, dtype=torch.float32, device=c.device)
        return dist[c]

    def _sample(self, n, device):
        import torch
        if self.sampler == 'uniform':
            s = torch.randint(0, self.C, (n, self.k), generator=self.gen)
        elif self.sampler == 'log_uniform':
            u = torch.rand((n, self.k), generator=self.gen)
            s = (torch.exp(u * torch.log(torch.tensor(self.C + 1.0))) - 1).long().clamp(0, self.C - 1)
        else:
            dist = torch.tensor(self.custom, dtype=torch.float32)
            s = torch.multinomial(dist, n * self.k, replacement=True, generator=self.gen)
            s = s.view(n, self.k)
        return s.to(device)

    def forward(self, x, label, sample_weight=None):
        import torch
        t = _u(x)
        lab = _u(label).long().reshape(t.shape[0], -1)
        neg = self._sample(t.shape[0], t.device)
        cls = torch.cat([lab, neg], 1)                                  # [N, T + k]
        logit = torch.einsum('nd,ncd->nc', t, self.weight._t[cls])
        if self.bias is not None:
            logit = logit + self.bias._t.reshape(-1)[cls]
        o = torch.sigmoid(logit)
        b = self.k * self._q(cls)
        nt = lab.shape[1]
        cost = -torch.log(o[:, :nt] / (o[:, :nt] + b[:, :nt])).sum(1) \
            - torch.log(b[:, nt:] / (o[:, nt:] + b[:, nt:])).sum(1)
        if sample_weight is not None:
            cost = cost * _u(sample_weight).reshape(-1)
        return Tensor(cost.unsqueeze(-1))


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None,
        num_neg_samples=None, name=None, sampler='uniform', custom_dist=None, seed=0,
        is_sparse=False):
    layer = _keep(_NCE(input.shape[-1], num_total_classes, num_neg_samples or 10, sampler,
                       custom_dist, seed, param_attr, bias_attr))
    return layer(input, label, sample_weight)


class _RowConv(_nn.Layer):
    """Lookahead row convolution (parity: paddle/fluid/operators/row_conv_op.cc):
    out[b, t] = Σ_{i=0..k} x[b, t+i] * W[i] (per feature), zero past the sequence end.
    Input is padded [B, T, D] (the reference's LoD form without LoD)."""

    def __init__(self, D, future_context_size, param_attr):
        super().__init__()
        self.weight = self.create_parameter([future_context_size + 1, D], param_attr)
        self.k = future_context_size

    def forward(self, x):
        import torch
        t = _u(x)
        T = t.shape[1]
        pad = torch.nn.functional.pad(t, (0, 0, 0, self.k))
        out = sum(pad[:, i:i + T] * self.weight._t[i] for i in range(self.k + 1))
        return Tensor(out)


def row_conv(input, future_context_size, param_attr=None, act=None):
    out = _keep(_RowConv(input.shape[-1], future_context_size, param_attr))(input)
    return getattr(F, act)(out) if act else out


from .control_flow import cond, while_loop, StaticRNN  # noqa: E402,F401


def case(pred_fn_pairs, default=None, name=None):
    """First true predicate's branch, else ``default`` — nested run-time ``cond`` ops."""
    pairs = list(pred_fn_pairs)
    if not pairs:
        return default() if default else None
    (pred, fn), rest = pairs[0], pairs[1:]
    if not rest and default is None:
        return fn()
    return cond(pred, fn, lambda: case(rest, default))


def switch_case(branch_index, branch_fns, default=None, name=None):
    from .. import equal, full
    items = list(branch_fns.items()) if isinstance(branch_fns, dict) else \
        (list(enumerate(branch_fns)) if not isinstance(branch_fns[0], (list, tuple))
         else list(branch_fns))
    pairs = [(equal(branch_index, full([1], k, branch_index.dtype)), fn) for k, fn in items]
    if default is None:
        default = items[-1][1]
        pairs = pairs[:-1]
    return case(pairs, default)


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    from .graph import py_func as pf
    return pf(func, x, out, backward_func, skip_vars_in_backward_input)


from .sequence_lod import (  # noqa: E402,F401
    sequence_conv, sequence_softmax, sequence_pool, sequence_concat, sequence_first_step,
    sequence_last_step, sequence_slice, sequence_expand, sequence_expand_as, sequence_pad,
    sequence_unpad, sequence_reshape, sequence_scatter, sequence_enumerate, sequence_reverse)
