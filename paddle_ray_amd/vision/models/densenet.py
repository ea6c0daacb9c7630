"""DenseNet-121/161/169/201/264 (parity: python/paddle/vision/models/densenet.py).

Each dense layer is BN-ReLU-conv1x1(bn_size*growth)-BN-ReLU-conv3x3(growth) and appends
its output to the running feature list; transitions halve channels and resolution."""
from ... import nn
from ...tensor import manipulation as M

_CFG = {121: (64, 32, [6, 12, 24, 16]), 161: (96, 48, [6, 12, 36, 24]),
        169: (64, 32, [6, 12, 32, 32]), 201: (64, 32, [6, 12, 48, 32]),
        264: (64, 32, [6, 12, 64, 48])}


class _DenseLayer(nn.Layer):
    def __init__(self, cin, growth, bn_size, dropout):
        super().__init__()
        self.norm1 = nn.BatchNorm2D(cin)
        self.conv1 = nn.Conv2D(cin, bn_size * growth, 1, bias_attr=False)
        self.norm2 = nn.BatchNorm2D(bn_size * growth)
        self.conv2 = nn.Conv2D(bn_size * growth, growth, 3, padding=1, bias_attr=False)
        self.relu = nn.ReLU()
        self.drop = nn.Dropout(dropout) if dropout > 0 else None

    def forward(self, x):
        y = self.conv1(self.relu(self.norm1(x)))
        y = self.conv2(self.relu(self.norm2(y)))
        if self.drop is not None:
            y = self.drop(y)
        return M.concat([x, y], axis=1)


class _Transition(nn.Sequential):
    def __init__(self, cin, cout):
        super().__init__(nn.BatchNorm2D(cin), nn.ReLU(), nn.Conv2D(cin, cout, 1, bias_attr=False),
                         nn.AvgPool2D(2, 2))


class DenseNet(nn.Layer):
    def __init__(self, layers=121, bn_size=4, dropout=0.0, num_classes=1000, with_pool=True):
        super().__init__()
        if layers not in _CFG:
            raise ValueError(f"supported layers are {sorted(_CFG)}, got {layers}")
        init_c, growth, blocks = _CFG[layers]
        self.num_classes, self.with_pool = num_classes, with_pool
        feats = [nn.Conv2D(3, init_c, 7, 2, 3, bias_attr=False), nn.BatchNorm2D(init_c),
                 nn.ReLU(), nn.MaxPool2D(3, 2, 1)]
        c = init_c
        for i, n in enumerate(blocks):
            for _ in range(n):
                feats.append(_DenseLayer(c, growth, bn_size, dropout))
                c += growth
            if i != len(blocks) - 1:
                feats.append(_Transition(c, c // 2))
                c //= 2
        feats += [nn.BatchNorm2D(c), nn.ReLU()]
        self.features = nn.Sequential(*feats)
        self.out_channels = c
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(c, num_classes)

    def forward(self, x):
        from ._blocks import classifier_head
        return classifier_head(self, self.features(x))


def _densenet(layers, pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return DenseNet(layers=layers, **kwargs)


def densenet121(pretrained=False, **kwargs):
    return _densenet(121, pretrained, **kwargs)


def densenet161(pretrained=False, **kwargs):
    return _densenet(161, pretrained, **kwargs)


def densenet169(pretrained=False, **kwargs):
    return _densenet(169, pretrained, **kwargs)


def densenet201(pretrained=False, **kwargs):
    return _densenet(201, pretrained, **kwargs)


def densenet264(pretrained=False, **kwargs):
    return _densenet(264, pretrained, **kwargs)
