"""paddle.sparse.nn (parity: python/paddle/sparse/nn/{layer,functional}).

Sparse COO tensors here are torch sparse tensors whose sparse dims are (N, D, H, W) and
whose dense dim is the channel (NDHWC, values [nnz, C]) -- the reference's layout for 3-D
point-cloud / voxel networks. Convolutions and max pooling run on the active sites only through
a rulebook (sparse/rulebook.py: gather - GEMM - scatter per kernel offset, O(nnz x kernel
volume)): a regular Conv3D activates every output site reached by an active input site, a
submanifold conv keeps exactly the input's active sites.
"""
import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _u
from ...nn.layer.layers import Layer
from ...nn import initializer as I


def _coo(x):
    t = _u(x)
    return t.coalesce() if t.layout == torch.sparse_coo else t.to_sparse_coo().coalesce()


def _like(t, values):
    return Tensor(torch.sparse_coo_tensor(t.indices(), values, t.shape).coalesce())


def _triple(v):
    return (v, v, v) if isinstance(v, int) else tuple(v)


def _from_dense(dense_ndhwc, active):
    """Sparse COO of ``dense`` at the boolean ``active`` [N, D, H, W] sites."""
    idx = active.nonzero().t()
    vals = dense_ndhwc[active]
    return Tensor(torch.sparse_coo_tensor(idx, vals, dense_ndhwc.shape).coalesce())


class _Functional:
    @staticmethod
    def relu(x, name=None):
        t = _coo(x)
        return _like(t, torch.relu(t.values()))

    @staticmethod
    def relu6(x, name=None):
        t = _coo(x)
        return _like(t, torch.clamp(t.values(), 0, 6))

    @staticmethod
    def leaky_relu(x, negative_slope=0.01, name=None):
        t = _coo(x)
        return _like(t, TF.leaky_relu(t.values(), negative_slope))

    @staticmethod
    def softmax(x, axis=-1, name=None):
        """Softmax over the stored entries of each row (missing entries are -inf)."""
        from ..ops import row_softmax
        t = _u(x)
        if axis not in (-1, t.dim() - 1):
            raise ValueError("sparse softmax supports the last axis only (as the reference)")
        return Tensor(row_softmax(t))

    @staticmethod
    def _conv(x, weight, bias, stride, padding, dilation, groups, subm):
        """Rulebook gather-GEMM-scatter on the active sites (sparse/rulebook.py)."""
        from ..rulebook import sparse_conv3d
        t = _coo(x)
        N, D, H, W = t.shape[:4]
        w = _u(weight)  # [kD, kH, kW, Cin/groups, Cout]
        out, oc, osp = sparse_conv3d(t.values(), t.indices().t(), N, (D, H, W), w,
                                     None if bias is None else _u(bias), stride, padding, dilation,
                                     groups, subm)
        return Tensor(torch.sparse_coo_tensor(oc.t(), out, (N,) + tuple(osp) + (w.shape[-1],)).coalesce())

    @staticmethod
    def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
               data_format='NDHWC', name=None):
        return _Functional._conv(x, weight, bias, stride, padding, dilation, groups, False)

    @staticmethod
    def subm_conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                    data_format='NDHWC', key=None, name=None):
        return _Functional._conv(x, weight, bias, stride, padding, dilation, groups, True)

    @staticmethod
    def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False,
                   data_format='NDHWC', name=None):
        """Max over the ACTIVE sites of each window; windows without one stay inactive."""
        from ..rulebook import sparse_max_pool3d
        if ceil_mode:
            raise NotImplementedError("sparse max_pool3d: ceil_mode")
        t = _coo(x)
        N, D, H, W = t.shape[:4]
        out, oc, osp = sparse_max_pool3d(t.values(), t.indices().t(), N, (D, H, W), kernel_size, stride,
                                         _triple(padding))
        return Tensor(torch.sparse_coo_tensor(oc.t(), out, (N,) + tuple(osp) + (t.shape[-1],)).coalesce())

    @staticmethod
    def attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None,
                  name=None):
        """softmax(QK^T / sqrt(d)) V on the coordinates of ``sparse_mask`` ([B*H, S, S] CSR /
        COO) only: SDDMM, row softmax and SpMM over the stored entries (sparse/ops.py)."""
        from ..ops import attention
        kp = None if key_padding_mask is None else _u(key_padding_mask)
        am = None if attn_mask is None else _u(attn_mask)
        return Tensor(attention(_u(query), _u(key), _u(value), _u(sparse_mask), kp, am))


class ReLU(Layer):
    def forward(self, x):
        return _Functional.relu(x)


class ReLU6(Layer):
    def forward(self, x):
        return _Functional.relu6(x)


class LeakyReLU(Layer):
    def __init__(self, negative_slope=0.01, name=None):
        super().__init__()
        self._slope = negative_slope

    def forward(self, x):
        return _Functional.leaky_relu(x, self._slope)


class Softmax(Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__()
        self._axis = axis

    def forward(self, x):
        return _Functional.softmax(x, self._axis)


class _Conv3DBase(Layer):
    _subm = False

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, padding_mode='zeros', key=None, weight_attr=None, bias_attr=None,
                 data_format='NDHWC'):
        super().__init__()
        k = _triple(kernel_size)
        self._stride, self._padding, self._dilation, self._groups = stride, padding, dilation, \
            groups
        fan_in = in_channels // groups * k[0] * k[1] * k[2]
        self.weight = self.create_parameter(
            [k[0], k[1], k[2], in_channels // groups, out_channels], attr=weight_attr,
            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = None if bias_attr is False else self.create_parameter(
            [out_channels], attr=bias_attr, is_bias=True)

    def forward(self, x):
        fn = _Functional.subm_conv3d if self._subm else _Functional.conv3d
        return fn(x, self.weight, self.bias, self._stride, self._padding, self._dilation,
                  self._groups)


class Conv3D(_Conv3DBase):
    pass


class SubmConv3D(_Conv3DBase):
    _subm = True


class MaxPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format='NDHWC', name=None):
        super().__init__()
        self._k, self._s, self._p, self._ceil = kernel_size, stride, padding, ceil_mode

    def forward(self, x):
        return _Functional.max_pool3d(x, self._k, self._s, self._p, self._ceil)


class BatchNorm(Layer):
    """BatchNorm over the channel of the stored values ([nnz, C]) of a sparse tensor."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None,
                 bias_attr=None, data_format='NDHWC', use_global_stats=None, name=None):
        super().__init__()
        from ...nn import BatchNorm1D
        self._bn = BatchNorm1D(num_features, momentum, epsilon, weight_attr, bias_attr)

    def forward(self, x):
        t = _coo(x)
        return _like(t, _u(self._bn(Tensor(t.values()))))


class SyncBatchNorm(BatchNorm):
    """Cross-rank statistics come from the dense SyncBatchNorm when a process group is up."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None,
                 bias_attr=None, data_format='NDHWC', name=None):
        Layer.__init__(self)
        from ...nn import SyncBatchNorm as _Sync
        self._bn = _Sync(num_features, momentum, epsilon, weight_attr, bias_attr, 'NCL')


from . import functional  # noqa: E402,F401
