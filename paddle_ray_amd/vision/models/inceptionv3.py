"""Inception-v3 (parity: python/paddle/vision/models/inceptionv3.py), 299x299 input.

Blocks A (5x5 + double 3x3), B (grid reduction), C (factorized 7x7), D (reduction with
7x7), E (expanded 3x3 splits); every conv is conv-BN(eps 1e-3)-ReLU."""
from ... import nn
from ...tensor import manipulation as M
from ._blocks import ConvBNAct


def _c(cin, cout, k, stride=1, padding=None):
    return ConvBNAct(cin, cout, k, stride, padding, act='relu', bn_eps=1e-3)


def _cat(xs):
    return M.concat(xs, axis=1)


class _A(nn.Layer):
    def __init__(self, cin, pool_c):
        super().__init__()
        self.b1 = _c(cin, 64, 1)
        self.b5 = nn.Sequential(_c(cin, 48, 1), _c(48, 64, 5))
        self.b3 = nn.Sequential(_c(cin, 64, 1), _c(64, 96, 3), _c(96, 96, 3))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1, exclusive=False), _c(cin, pool_c, 1))

    def forward(self, x):
        return _cat([self.b1(x), self.b5(x), self.b3(x), self.bp(x)])


class _B(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b3 = _c(cin, 384, 3, 2, 0)
        self.bd = nn.Sequential(_c(cin, 64, 1), _c(64, 96, 3), _c(96, 96, 3, 2, 0))
        self.bp = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return _cat([self.b3(x), self.bd(x), self.bp(x)])


class _C(nn.Layer):
    def __init__(self, cin, c7):
        super().__init__()
        self.b1 = _c(cin, 192, 1)
        self.b7 = nn.Sequential(_c(cin, c7, 1), _c(c7, c7, (1, 7)), _c(c7, 192, (7, 1)))
        self.bd = nn.Sequential(_c(cin, c7, 1), _c(c7, c7, (7, 1)), _c(c7, c7, (1, 7)),
                                _c(c7, c7, (7, 1)), _c(c7, 192, (1, 7)))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1, exclusive=False), _c(cin, 192, 1))

    def forward(self, x):
        return _cat([self.b1(x), self.b7(x), self.bd(x), self.bp(x)])


class _D(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b3 = nn.Sequential(_c(cin, 192, 1), _c(192, 320, 3, 2, 0))
        self.b7 = nn.Sequential(_c(cin, 192, 1), _c(192, 192, (1, 7)), _c(192, 192, (7, 1)),
                                _c(192, 192, 3, 2, 0))
        self.bp = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return _cat([self.b3(x), self.b7(x), self.bp(x)])


class _E(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b1 = _c(cin, 320, 1)
        self.b3 = _c(cin, 384, 1)
        self.b3a, self.b3b = _c(384, 384, (1, 3)), _c(384, 384, (3, 1))
        self.bd = nn.Sequential(_c(cin, 448, 1), _c(448, 384, 3))
        self.bda, self.bdb = _c(384, 384, (1, 3)), _c(384, 384, (3, 1))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1, exclusive=False), _c(cin, 192, 1))

    def forward(self, x):
        y3 = self.b3(x)
        yd = self.bd(x)
        return _cat([self.b1(x), self.b3a(y3), self.b3b(y3), self.bda(yd), self.bdb(yd),
                     self.bp(x)])


class InceptionV3(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.stem = nn.Sequential(_c(3, 32, 3, 2, 0), _c(32, 32, 3, 1, 0), _c(32, 64, 3),
                                  nn.MaxPool2D(3, 2), _c(64, 80, 1), _c(80, 192, 3, 1, 0),
                                  nn.MaxPool2D(3, 2))
        self.blocks = nn.Sequential(_A(192, 32), _A(256, 64), _A(288, 64), _B(288),
                                    _C(768, 128), _C(768, 160), _C(768, 160), _C(768, 192),
                                    _D(768), _E(1280), _E(2048))
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.drop = nn.Dropout(0.2)
            self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        if self.with_pool:
            x = self.pool(x)
        if self.num_classes > 0:
            x = self.fc(self.drop(x.flatten(1)))
        return x


def inception_v3(pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return InceptionV3(**kwargs)
