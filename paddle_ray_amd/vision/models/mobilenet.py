"""MobileNetV1/V2 (parity: python/paddle/vision/models/mobilenetv1.py, mobilenetv2.py)."""
from ... import nn


class ConvBNLayer(nn.Layer):
    def __init__(self, cin, cout, k, stride, padding, groups=1, act=True):
        super().__init__()
        self._conv = nn.Conv2D(cin, cout, k, stride, padding, groups=groups, bias_attr=False)
        self._bn = nn.BatchNorm2D(cout)
        self._act = nn.ReLU6() if act == 'relu6' else (nn.ReLU() if act else None)

    def forward(self, x):
        x = self._bn(self._conv(x))
        return self._act(x) if self._act is not None else x


class MobileNetV1(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        s = lambda c: int(c * scale)  # noqa: E731
        cfg = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1),
               (256, 512, 2)] + [(512, 512, 1)] * 5 + [(512, 1024, 2), (1024, 1024, 1)]
        layers = [ConvBNLayer(3, s(32), 3, 2, 1)]
        for cin, cout, st in cfg:
            layers += [ConvBNLayer(s(cin), s(cin), 3, st, 1, groups=s(cin)),
                       ConvBNLayer(s(cin), s(cout), 1, 1, 0)]
        self.features = nn.Sequential(*layers)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(s(1024), num_classes)

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.fc(x.flatten(1))
        return x


class InvertedResidual(nn.Layer):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNLayer(inp, hidden, 1, 1, 0, act='relu6'))
        layers += [ConvBNLayer(hidden, hidden, 3, stride, 1, groups=hidden, act='relu6'),
                   ConvBNLayer(hidden, oup, 1, 1, 0, act=False)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1],
               [6, 160, 3, 2], [6, 320, 1, 1]]
        inp = int(32 * scale)
        self.last_channel = int(1280 * max(1.0, scale))
        feats = [ConvBNLayer(3, inp, 3, 2, 1, act='relu6')]
        for t, c, n, s in cfg:
            out = int(c * scale)
            for i in range(n):
                feats.append(InvertedResidual(inp, out, s if i == 0 else 1, t))
                inp = out
        feats.append(ConvBNLayer(inp, self.last_channel, 1, 1, 0, act='relu6'))
        self.features = nn.Sequential(*feats)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(self.last_channel,
                                                                       num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.classifier(x.flatten(1))
        return x


def mobilenet_v1(pretrained=False, scale=1.0, **kw):
    return MobileNetV1(scale=scale, **kw)


def mobilenet_v2(pretrained=False, scale=1.0, **kw):
    return MobileNetV2(scale=scale, **kw)
