"""paddle.sparse.nn.functional (parity: python/paddle/sparse/nn/functional/__init__.py): the
functional forms of the sparse layers -- activations on the stored values, rulebook sparse /
submanifold 3-D convolution, 3-D max pooling and masked sparse attention."""
from . import _Functional as _F

__all__ = ['conv3d', 'subm_conv3d', 'max_pool3d', 'relu', 'relu6', 'leaky_relu', 'softmax', 'attention']

relu = _F.relu
relu6 = _F.relu6
leaky_relu = _F.leaky_relu
softmax = _F.softmax
conv3d = _F.conv3d
subm_conv3d = _F.subm_conv3d
max_pool3d = _F.max_pool3d
attention = _F.attention
_conv = _F._conv
