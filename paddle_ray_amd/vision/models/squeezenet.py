"""SqueezeNet 1.0 / 1.1 (parity: python/paddle/vision/models/squeezenet.py)."""
from ... import nn
from ...tensor import manipulation as M


class _Fire(nn.Layer):
    """squeeze 1x1 -> (expand 1x1 | expand 3x3) concatenated, all ReLU."""

    def __init__(self, cin, squeeze, e1, e3):
        super().__init__()
        self.squeeze = nn.Conv2D(cin, squeeze, 1)
        self.e1 = nn.Conv2D(squeeze, e1, 1)
        self.e3 = nn.Conv2D(squeeze, e3, 3, padding=1)
        self.relu = nn.ReLU()

    def forward(self, x):
        s = self.relu(self.squeeze(x))
        return M.concat([self.relu(self.e1(s)), self.relu(self.e3(s))], axis=1)


class SqueezeNet(nn.Layer):
    def __init__(self, version, num_classes=1000, with_pool=True):
        super().__init__()
        self.version, self.num_classes, self.with_pool = version, num_classes, with_pool
        pool = lambda: nn.MaxPool2D(3, 2, ceil_mode=True)  # noqa: E731
        if version == '1.0':
            layers = [nn.Conv2D(3, 96, 7, 2), nn.ReLU(), pool(), _Fire(96, 16, 64, 64),
                      _Fire(128, 16, 64, 64), _Fire(128, 32, 128, 128), pool(),
                      _Fire(256, 32, 128, 128), _Fire(256, 48, 192, 192),
                      _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), pool(),
                      _Fire(512, 64, 256, 256)]
        elif version == '1.1':
            layers = [nn.Conv2D(3, 64, 3, 2), nn.ReLU(), pool(), _Fire(64, 16, 64, 64),
                      _Fire(128, 16, 64, 64), pool(), _Fire(128, 32, 128, 128),
                      _Fire(256, 32, 128, 128), pool(), _Fire(256, 48, 192, 192),
                      _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256),
                      _Fire(512, 64, 256, 256)]
        else:
            raise ValueError("version must be '1.0' or '1.1'")
        self.features = nn.Sequential(*layers)
        if num_classes > 0:
            self.drop = nn.Dropout(0.5)
            self.final_conv = nn.Conv2D(512, num_classes, 1)
            self.relu = nn.ReLU()
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)

    def forward(self, x):
        x = self.features(x)
        if self.num_classes > 0:
            x = self.relu(self.final_conv(self.drop(x)))
        if self.with_pool:
            x = self.pool(x)
            x = x.flatten(1)
        return x


def squeezenet1_0(pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return SqueezeNet('1.0', **kwargs)


def squeezenet1_1(pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return SqueezeNet('1.1', **kwargs)
