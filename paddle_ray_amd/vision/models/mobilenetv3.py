"""MobileNetV3 small / large (parity: python/paddle/vision/models/mobilenetv3.py)."""
from ... import nn
from ._blocks import ConvBNAct, make_divisible

# (kernel, expanded, out, squeeze-excite, activation, stride)
_LARGE = [(3, 16, 16, False, 'relu', 1), (3, 64, 24, False, 'relu', 2),
          (3, 72, 24, False, 'relu', 1), (5, 72, 40, True, 'relu', 2),
          (5, 120, 40, True, 'relu', 1), (5, 120, 40, True, 'relu', 1),
          (3, 240, 80, False, 'hardswish', 2), (3, 200, 80, False, 'hardswish', 1),
          (3, 184, 80, False, 'hardswish', 1), (3, 184, 80, False, 'hardswish', 1),
          (3, 480, 112, True, 'hardswish', 1), (3, 672, 112, True, 'hardswish', 1),
          (5, 672, 160, True, 'hardswish', 2), (5, 960, 160, True, 'hardswish', 1),
          (5, 960, 160, True, 'hardswish', 1)]
_SMALL = [(3, 16, 16, True, 'relu', 2), (3, 72, 24, False, 'relu', 2),
          (3, 88, 24, False, 'relu', 1), (5, 96, 40, True, 'hardswish', 2),
          (5, 240, 40, True, 'hardswish', 1), (5, 240, 40, True, 'hardswish', 1),
          (5, 120, 48, True, 'hardswish', 1), (5, 144, 48, True, 'hardswish', 1),
          (5, 288, 96, True, 'hardswish', 2), (5, 576, 96, True, 'hardswish', 1),
          (5, 576, 96, True, 'hardswish', 1)]


class SqueezeExcitation(nn.Layer):
    def __init__(self, c, squeeze_c):
        super().__init__()
        self.pool = nn.AdaptiveAvgPool2D(1)
        self.fc1 = nn.Conv2D(c, squeeze_c, 1)
        self.fc2 = nn.Conv2D(squeeze_c, c, 1)
        self.relu = nn.ReLU()
        self.gate = nn.Hardsigmoid()

    def forward(self, x):
        return x * self.gate(self.fc2(self.relu(self.fc1(self.pool(x)))))


class InvertedResidualV3(nn.Layer):
    def __init__(self, cin, k, exp, cout, se, act, stride):
        super().__init__()
        self.use_res = stride == 1 and cin == cout
        layers = []
        if exp != cin:
            layers.append(ConvBNAct(cin, exp, 1, act=act))
        layers.append(ConvBNAct(exp, exp, k, stride, groups=exp, act=act))
        if se:
            layers.append(SqueezeExcitation(exp, make_divisible(exp // 4)))
        layers.append(ConvBNAct(exp, cout, 1, act=None))
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        y = self.block(x)
        return x + y if self.use_res else y


class MobileNetV3(nn.Layer):
    def __init__(self, config, last_channel, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        s = lambda c: make_divisible(c * scale)  # noqa: E731
        layers = [ConvBNAct(3, s(16), 3, 2, act='hardswish')]
        cin = s(16)
        for k, exp, out, se, act, st in config:
            layers.append(InvertedResidualV3(cin, k, s(exp), s(out), se, act, st))
            cin = s(out)
        last_conv = s(6 * config[-1][2])
        layers.append(ConvBNAct(cin, last_conv, 1, act='hardswish'))
        self.features = nn.Sequential(*layers)
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(last_conv, last_channel), nn.Hardswish(),
                                            nn.Dropout(0.2), nn.Linear(last_channel, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool(x)
        if self.num_classes > 0:
            x = self.classifier(x.flatten(1))
        return x


class MobileNetV3Small(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__(_SMALL, make_divisible(1024 * scale), scale, num_classes, with_pool)


class MobileNetV3Large(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__(_LARGE, make_divisible(1280 * scale), scale, num_classes, with_pool)


def mobilenet_v3_small(pretrained=False, scale=1.0, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return MobileNetV3Small(scale=scale, **kwargs)


def mobilenet_v3_large(pretrained=False, scale=1.0, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return MobileNetV3Large(scale=scale, **kwargs)
