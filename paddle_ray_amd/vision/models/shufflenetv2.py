"""ShuffleNetV2 x0.25 ... x2.0 and the swish variant (parity:
python/paddle/vision/models/shufflenetv2.py)."""
from ... import nn
from ...tensor import manipulation as M
from ._blocks import ConvBNAct

_CHANNELS = {0.25: [24, 24, 48, 96, 512], 0.33: [24, 32, 64, 128, 512],
             0.5: [24, 48, 96, 192, 1024], 1.0: [24, 116, 232, 464, 1024],
             1.5: [24, 176, 352, 704, 1024], 2.0: [24, 224, 488, 976, 2048]}


def channel_shuffle(x, groups):
    n, c, h, w = x.shape
    return M.reshape(M.transpose(M.reshape(x, [n, groups, c // groups, h, w]), [0, 2, 1, 3, 4]),
                     [n, c, h, w])


class _ShuffleUnit(nn.Layer):
    def __init__(self, cin, cout, stride, act):
        super().__init__()
        self.stride = stride
        mid = cout // 2
        if stride == 1:
            b_in = cin // 2
        else:
            b_in = cin
            self.branch1 = nn.Sequential(ConvBNAct(cin, cin, 3, stride, groups=cin, act=None),
                                         ConvBNAct(cin, mid, 1, act=act))
        self.branch2 = nn.Sequential(ConvBNAct(b_in, mid, 1, act=act),
                                     ConvBNAct(mid, mid, 3, stride, groups=mid, act=None),
                                     ConvBNAct(mid, mid, 1, act=act))

    def forward(self, x):
        if self.stride == 1:
            a, b = M.split(x, 2, axis=1)
            out = M.concat([a, self.branch2(b)], axis=1)
        else:
            out = M.concat([self.branch1(x), self.branch2(x)], axis=1)
        return channel_shuffle(out, 2)


class ShuffleNetV2(nn.Layer):
    def __init__(self, scale=1.0, act='relu', num_classes=1000, with_pool=True):
        super().__init__()
        if scale not in _CHANNELS:
            raise ValueError(f"scale must be one of {sorted(_CHANNELS)}")
        ch = _CHANNELS[scale]
        self.num_classes, self.with_pool = num_classes, with_pool
        layers = [ConvBNAct(3, ch[0], 3, 2, act=act), nn.MaxPool2D(3, 2, 1)]
        cin = ch[0]
        for reps, cout in zip([4, 8, 4], ch[1:4]):
            for i in range(reps):
                layers.append(_ShuffleUnit(cin, cout, 2 if i == 0 else 1, act))
                cin = cout
        layers.append(ConvBNAct(cin, ch[4], 1, act=act))
        self.features = nn.Sequential(*layers)
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(ch[4], num_classes)

    def forward(self, x):
        from ._blocks import classifier_head
        return classifier_head(self, self.features(x))


def _shufflenet(scale, act='relu', pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return ShuffleNetV2(scale=scale, act=act, **kwargs)


def shufflenet_v2_x0_25(pretrained=False, **kwargs):
    return _shufflenet(0.25, pretrained=pretrained, **kwargs)


def shufflenet_v2_x0_33(pretrained=False, **kwargs):
    return _shufflenet(0.33, pretrained=pretrained, **kwargs)


def shufflenet_v2_x0_5(pretrained=False, **kwargs):
    return _shufflenet(0.5, pretrained=pretrained, **kwargs)


def shufflenet_v2_x1_0(pretrained=False, **kwargs):
    return _shufflenet(1.0, pretrained=pretrained, **kwargs)


def shufflenet_v2_x1_5(pretrained=False, **kwargs):
    return _shufflenet(1.5, pretrained=pretrained, **kwargs)


def shufflenet_v2_x2_0(pretrained=False, **kwargs):
    return _shufflenet(2.0, pretrained=pretrained, **kwargs)


def shufflenet_v2_swish(pretrained=False, **kwargs):
    return _shufflenet(1.0, act='swish', pretrained=pretrained, **kwargs)
