"""Normalization layers (parity: python/paddle/nn/layer/norm.py).

LayerNorm/RMSNorm run the gfx950 row kernels; BatchNorm uses MIOpen via
PyTorch-ROCm (channels-first) with paddle's momentum convention
(running = momentum * running + (1 - momentum) * batch).
"""
import numpy as np
import torch

from ...framework.core import Tensor, _u
from .. import functional as F
from .. import initializer as I
from .layers import Layer


class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-05, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = [normalized_shape]
        self._normalized_shape = list(normalized_shape)
        self._epsilon = epsilon
        n = int(np.prod(normalized_shape))
        self.weight = self.create_parameter([n], weight_attr, default_initializer=I.Constant(1.0)) \
            if weight_attr is not False else None
        self.bias = self.create_parameter([n], bias_attr, is_bias=True) if bias_attr is not False \
            else None

    def forward(self, x):
        return F.layer_norm(x, self._normalized_shape, self.weight, self.bias, self._epsilon)

    def extra_repr(self):
        return f'normalized_shape={self._normalized_shape}, epsilon={self._epsilon}'


class RMSNorm(Layer):
    def __init__(self, hidden_size, epsilon=1e-6, weight_attr=None, name=None):
        super().__init__()
        self._epsilon = epsilon
        self.weight = self.create_parameter([hidden_size], weight_attr,
                                            default_initializer=I.Constant(1.0))

    def forward(self, x):
        return F.rms_norm(x, self.weight, self._epsilon)


class _BatchNormBase(Layer):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format='NCHW', use_global_stats=None, name=None):
        super().__init__()
        self._num_features, self._momentum, self._epsilon = num_features, momentum, epsilon
        self._data_format = data_format
        self._use_global_stats = use_global_stats
        self.weight = self.create_parameter([num_features], weight_attr,
                                            default_initializer=I.Constant(1.0)) \
            if weight_attr is not False else None
        self.bias = self.create_parameter([num_features], bias_attr, is_bias=True) \
            if bias_attr is not False else None
        dt = torch.float32
        dev = self.weight._t.device if self.weight is not None else None
        self.register_buffer('_mean', Tensor(torch.zeros(num_features, dtype=dt, device=dev)))
        self.register_buffer('_variance', Tensor(torch.ones(num_features, dtype=dt, device=dev)))

    def forward(self, x):
        training = self.training and not self._use_global_stats
        return F.batch_norm(x, self._mean, self._variance, self.weight, self.bias, training,
                            self._momentum, self._epsilon, self._data_format)

    def extra_repr(self):
        return f'num_features={self._num_features}, momentum={self._momentum}, epsilon={self._epsilon}'


class BatchNorm(_BatchNormBase):
    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-05,
                 param_attr=None, bias_attr=None, dtype='float32', data_layout='NCHW',
                 in_place=False, moving_mean_name=None, moving_variance_name=None,
                 do_model_average_for_mean_and_var=True, use_global_stats=False,
                 trainable_statistics=False):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout,
                         use_global_stats)
        self._act = act

    def forward(self, x):
        out = super().forward(x)
        if self._act:
            out = getattr(F, self._act)(out)
        return out


class BatchNorm1D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format='NCL', use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format,
                         use_global_stats)


class BatchNorm2D(_BatchNormBase):
    pass


class BatchNorm3D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format='NCDHW', use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format,
                         use_global_stats)


class SyncBatchNorm(_BatchNormBase):
    """Cross-rank BN: batch statistics all-reduced over the default group (RCCL)."""

    def forward(self, x):
        import torch.distributed as dist
        if not (self.training and dist.is_available() and dist.is_initialized() and
                dist.get_world_size() > 1):
            return super().forward(x)
        t = _u(x)
        cl = self._data_format in ('NHWC', 'NLC', 'NDHWC')
        if cl:
            t = t.movedim(-1, 1)
        dims = [0] + list(range(2, t.dim()))
        n = torch.tensor([float(t.numel() // t.shape[1])], device=t.device)
        s = t.float().sum(dims)
        ss = (t.float() ** 2).sum(dims)
        st = torch.cat([s, ss, n])
        from ...distributed.collective import _all_reduce_autograd
        st = _all_reduce_autograd(st)
        C = t.shape[1]
        cnt = st[-1]
        mean = st[:C] / cnt
        var = st[C:2 * C] / cnt - mean ** 2
        with torch.no_grad():
            m = self._momentum
            self._mean._t.mul_(m).add_(mean.detach(), alpha=1 - m)
            self._variance._t.mul_(m).add_(var.detach() * cnt / (cnt - 1).clamp_min(1), alpha=1 - m)
        shp = [1, C] + [1] * (t.dim() - 2)
        out = (t.float() - mean.view(shp)) * torch.rsqrt(var.view(shp) + self._epsilon)
        if self.weight is not None:
            out = out * self.weight._t.float().view(shp) + self.bias._t.float().view(shp)
        out = out.to(t.dtype)
        if cl:
            out = out.movedim(1, -1)
        return Tensor(out)

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        out = layer
        if isinstance(layer, _BatchNormBase) and not isinstance(layer, SyncBatchNorm):
            out = SyncBatchNorm(layer._num_features, layer._momentum, layer._epsilon,
                                data_format=layer._data_format)
            out.weight, out.bias = layer.weight, layer.bias
            out._buffers['_mean'], out._buffers['_variance'] = layer._mean, layer._variance
        for n, sub in layer.named_children():
            out.add_sublayer(n, cls.convert_sync_batchnorm(sub))
        return out


class _InstanceNormBase(Layer):
    def __init__(self, num_features, epsilon=1e-05, momentum=0.9, weight_attr=None, bias_attr=None,
                 data_format='NCHW', name=None):
        super().__init__()
        self._epsilon = epsilon
        self.scale = self.create_parameter([num_features], weight_attr,
                                           default_initializer=I.Constant(1.0)) \
            if weight_attr is not False else None
        self.bias = self.create_parameter([num_features], bias_attr, is_bias=True) \
            if bias_attr is not False else None

    def forward(self, x):
        return F.instance_norm(x, weight=self.scale, bias=self.bias, eps=self._epsilon)


class InstanceNorm1D(_InstanceNormBase):
    pass


class InstanceNorm2D(_InstanceNormBase):
    pass


class InstanceNorm3D(_InstanceNormBase):
    pass


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format='NCHW', name=None):
        super().__init__()
        self._num_groups, self._epsilon, self._data_format = num_groups, epsilon, data_format
        self.weight = self.create_parameter([num_channels], weight_attr,
                                            default_initializer=I.Constant(1.0)) \
            if weight_attr is not False else None
        self.bias = self.create_parameter([num_channels], bias_attr, is_bias=True) \
            if bias_attr is not False else None

    def forward(self, x):
        return F.group_norm(x, self._num_groups, self._epsilon, self.weight, self.bias,
                            self._data_format)


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=0.0001, beta=0.75, k=1.0, data_format='NCHW', name=None):
        super().__init__()
        self.args = (size, alpha, beta, k, data_format)

    def forward(self, x):
        return F.local_response_norm(x, *self.args)


class SpectralNorm(Layer):
    def __init__(self, weight_shape, dim=0, power_iters=1, eps=1e-12, dtype='float32'):
        super().__init__()
        self._dim, self._power_iters, self._eps = dim, power_iters, eps
        h = weight_shape[dim]
        w = int(np.prod(weight_shape)) // h
        self.weight_u = self.create_parameter([h], default_initializer=I.Normal(0, 1))
        self.weight_v = self.create_parameter([w], default_initializer=I.Normal(0, 1))
        self.weight_u.stop_gradient = True
        self.weight_v.stop_gradient = True

    def forward(self, weight):
        w = _u(weight)
        mat = w.movedim(self._dim, 0).reshape(w.shape[self._dim], -1)
        u, v = self.weight_u._t, self.weight_v._t
        with torch.no_grad():
            for _ in range(self._power_iters):
                v.copy_(torch.nn.functional.normalize(mat.t() @ u, dim=0, eps=self._eps))
                u.copy_(torch.nn.functional.normalize(mat @ v, dim=0, eps=self._eps))
        sigma = u @ mat @ v
        return Tensor(w / sigma)
