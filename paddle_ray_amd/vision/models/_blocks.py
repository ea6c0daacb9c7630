"""Shared conv building blocks for the vision model zoo."""
from ... import nn


def make_divisible(v, divisor=8, min_value=None):
    """Round a channel count to a multiple of ``divisor`` without dropping >10%."""
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


_ACTS = {'relu': nn.ReLU, 'relu6': nn.ReLU6, 'hardswish': nn.Hardswish, 'swish': nn.Swish,
         None: None}


class ConvBNAct(nn.Layer):
    """conv (no bias) -> BatchNorm -> optional activation; 'same' padding by default."""

    def __init__(self, cin, cout, k, stride=1, padding=None, groups=1, act='relu',
                 bn_eps=1e-5):
        super().__init__()
        if padding is None:
            padding = ((k[0] - 1) // 2, (k[1] - 1) // 2) if isinstance(k, (tuple, list)) \
                else (k - 1) // 2
        self.conv = nn.Conv2D(cin, cout, k, stride, padding, groups=groups, bias_attr=False)
        self.bn = nn.BatchNorm2D(cout, epsilon=bn_eps)
        a = _ACTS[act]
        self.act = a() if a is not None else None

    def forward(self, x):
        x = self.bn(self.conv(x))
        return self.act(x) if self.act is not None else x


def classifier_head(layer, x):
    """Shared tail: optional global pool, then optional fc on the flattened features."""
    if layer.with_pool:
        x = layer.pool(x)
    if layer.num_classes > 0:
        x = layer.fc(x.flatten(1))
    return x
